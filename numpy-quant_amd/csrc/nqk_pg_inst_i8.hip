// k_pg instantiations, ViT-Base int8: QKV (+ 8-bit saturating form), FFN-up + GELU (filtered chain and table) (nqk_pgemm_kernel.h; one file per group so the library builds in
// parallel).
#include "nqk_pgemm_kernel.h"

namespace nqk {
bool pg_dispatch_i8(int key, const PgArgs& x) {
  switch (key) {
    NQK_PG_CASE(PG_QKV, 12, true, false, true, 1)
    NQK_PG_CASE(PG_QKV, 12, true, false, false, 1)
    NQK_PG_CASE(PG_GELU, 12, true, false, false, 1)
    NQK_PG_CASE(PG_GLUT, 12, true, false, false, 1)
    NQK_PG_CASE(PG_GLUT1, 12, true, false, false, 1)
    default:
      return false;
  }
}
}  // namespace nqk
