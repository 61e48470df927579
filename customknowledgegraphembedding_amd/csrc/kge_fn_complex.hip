// Instantiates the fused scoring kernels of one score function (KGE_COMPLEX); see kge_device.h.
#include "kge_device.h"

namespace kge_impl {
int launch_complex(const ScoreParams& p, int kind, hipStream_t st, int blocks, bool ch, int V, int G) {
    return launch_fn_tmpl<KGE_COMPLEX>(p, kind, st, blocks, ch, V, G);
}
}  // namespace kge_impl
