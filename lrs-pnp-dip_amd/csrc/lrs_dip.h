// Internal definitions shared by the DIP kernels (dip_kernels.hip) and the engine (dipnet.hip).
#pragma once
#include "lrs_common.h"

namespace lrs {

// Geometry of one conv: source [Cin][Hs][Ws] -> (optional nearest x2 upsample) [Hu][Wu]
// -> pad (reflect / zero) -> k x k conv with stride -> [Cout][Ho][Wo].
struct ConvGeom {
    int Cin, Hs, Ws, up, Hu, Wu, pad, pad_mode, k, stride, Ho, Wo;
    // host-side mode, fixed when the geometry is made (lrs_dip_opts): the GEMM arithmetic of the
    // explicit / 1x1 products, and the effective kernel size of the upsampled data gradient (0 = off)
    int prec, ke;
};

struct SnConv {
    const float *W;   // W_bar [rows][cols]
    float *Wn;        // W_bar / scale (written by k_sn_apply)
    int rows, cols;
};

}  // namespace lrs
