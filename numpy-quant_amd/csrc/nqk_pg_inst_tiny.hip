// k_pg instantiations, K = 192 (ViT-Ti/16) (nqk_pgemm_kernel.h; one file per group so the library builds in
// parallel).
#include "nqk_pgemm_kernel.h"

namespace nqk {
bool pg_dispatch_tiny(int key, const PgArgs& x) {
  switch (key) {
    NQK_PG_CASE(PG_QKV, 3, true, false, true, 1)
    NQK_PG_CASE(PG_QKV, 3, true, false, false, 1)
    NQK_PG_CASE(PG_GELU, 3, true, false, false, 1)
    NQK_PG_CASE(PG_GLUT, 3, true, false, false, 1)
    NQK_PG_CASE(PG_GLUT1, 3, true, false, false, 1)
    // 64-row tiles (WM = 0)
    NQK_PG_CASE(PG_QKV, 3, true, false, true, 0)
    NQK_PG_CASE(PG_QKV, 3, true, false, false, 0)
    NQK_PG_CASE(PG_GELU, 3, true, false, false, 0)
    NQK_PG_CASE(PG_GLUT, 3, true, false, false, 0)
    NQK_PG_CASE(PG_GLUT1, 3, true, false, false, 0)
    NQK_PG_CASE(PG_RESID, 3, true, false, false, 1)
    NQK_PG_CASE(PG_RESID, 3, false, false, false, 1)
    // the weight panel resident (RB)
    NQK_PG_CASE_RB(PG_QKV, 3, true, false, true, 1, true)
    NQK_PG_CASE_RB(PG_QKV, 3, true, false, false, 1, true)
    NQK_PG_CASE_RB(PG_GELU, 3, true, false, false, 1, true)
    NQK_PG_CASE_RB(PG_GLUT, 3, true, false, false, 1, true)
    NQK_PG_CASE_RB(PG_GLUT1, 3, true, false, false, 1, true)
    NQK_PG_CASE_RB(PG_GLUT, 3, true, false, false, 2, true)
    NQK_PG_CASE_RB(PG_GLUT1, 3, true, false, false, 2, true)
    default:
      return false;
  }
}
}  // namespace nqk
