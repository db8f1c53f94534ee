// k_pg instantiations, int4 nibble-packed weights (BASELINE configs[4]) (nqk_pgemm_kernel.h; one file per group so the library builds in
// parallel).
#include "nqk_pgemm_kernel.h"

namespace nqk {
bool pg_dispatch_i4(int key, const PgArgs& x) {
  switch (key) {
    NQK_PG_CASE(PG_QKV, 12, true, true, false, 1)
    NQK_PG_CASE(PG_GELU, 12, true, true, false, 1)
    NQK_PG_CASE(PG_GLUT, 12, true, true, false, 1)
    NQK_PG_CASE(PG_GLUT1, 12, true, true, false, 1)
    NQK_PG_CASE(PG_RESID, 12, true, true, false, 1)
    NQK_PG_CASE(PG_RESID, 12, false, true, false, 1)
    NQK_PG_CASE(PG_RESID, 48, true, true, false, 1)
    NQK_PG_CASE(PG_RESID, 48, false, true, false, 1)
    default:
      return false;
  }
}
}  // namespace nqk
