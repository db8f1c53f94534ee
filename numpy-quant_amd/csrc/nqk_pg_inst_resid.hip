// k_pg instantiations, int8 residual epilogues (attention output projection K = 768, FFN-down K = 3072) (nqk_pgemm_kernel.h; one file per group so the library builds in
// parallel).
#include "nqk_pgemm_kernel.h"

namespace nqk {
bool pg_dispatch_resid(int key, const PgArgs& x) {
  switch (key) {
    NQK_PG_CASE(PG_RESID, 12, true, false, false, 1)
    NQK_PG_CASE(PG_RESID, 12, false, false, false, 1)
    NQK_PG_CASE(PG_RESID, 48, true, false, false, 1)
    NQK_PG_CASE(PG_RESID, 48, false, false, false, 1)
    default:
      return false;
  }
}
}  // namespace nqk
