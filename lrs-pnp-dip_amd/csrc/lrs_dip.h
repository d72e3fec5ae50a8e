// Internal definitions shared by the DIP kernels (dip_kernels.hip) and the engine (dipnet.hip).
#pragma once
#include "lrs_common.h"

namespace lrs {

// Geometry of one conv: source [Cin][Hs][Ws] -> (optional nearest x2 upsample) [Hu][Wu]
// -> pad (reflect / zero) -> k x k conv with stride -> [Cout][Ho][Wo].
struct ConvGeom {
    int Cin, Hs, Ws, up, Hu, Wu, pad, pad_mode, k, stride, Ho, Wo;
};

struct SnConv {
    const float *W;   // W_bar [rows][cols]
    float *Wn;        // W_bar / scale (written by k_sn_apply)
    int rows, cols;
};

}  // namespace lrs
