// wk_fused_xdl.hip -- the fused kernel for the bf16-family convolutions
// (conv_mode 1 = bf16, config 4; 2 = split bf16): wk_fused.hip compiled again
// with the front-end's complex arithmetic as scalar fp32 pairs (WK_FE_SCALAR,
// wk_common.h).  It defines wk::launch_fused_xdl only; wk::launch_fused
// (wk_fused.hip) calls it for those modes.  Empty in diagnostic builds
// (WK_FUSED_ONE_TU).
#define WK_FE_SCALAR 1
#define WK_FUSED_XDL_TU 1
#include "wk_fused.hip"
