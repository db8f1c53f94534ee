// k_pg instantiations, 256 x 256 tiles (WM = 2: one 512-thread workgroup per CU, B shared by the two row halves), int8 (nqk_pgemm_kernel.h; one file per group so the library builds in
// parallel).
#include "nqk_pgemm_kernel.h"

namespace nqk {
bool pg_dispatch_wm2(int key, const PgArgs& x) {
  switch (key) {
    NQK_PG_CASE(PG_QKV, 12, true, false, true, 2)
    NQK_PG_CASE(PG_QKV, 12, true, false, false, 2)
    NQK_PG_CASE(PG_GELU, 12, true, false, false, 2)
    NQK_PG_CASE(PG_GLUT, 12, true, false, false, 2)
    NQK_PG_CASE(PG_GLUT1, 12, true, false, false, 2)
    NQK_PG_CASE(PG_GLUT, 3, true, false, false, 2)
    NQK_PG_CASE(PG_GLUT1, 3, true, false, false, 2)
    NQK_PG_CASE(PG_RESID, 12, true, false, false, 2)
    NQK_PG_CASE(PG_RESID, 12, false, false, false, 2)
    NQK_PG_CASE(PG_RESID, 48, true, false, false, 2)
    NQK_PG_CASE(PG_RESID, 48, false, false, false, 2)
    default:
      return false;
  }
}
}  // namespace nqk
