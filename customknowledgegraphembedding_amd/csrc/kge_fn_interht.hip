// Instantiates the fused scoring kernels of one score function (KGE_INTERHT); see kge_device.h.
#include "kge_device.h"

namespace kge_impl {
int launch_interht(const ScoreParams& p, int kind, hipStream_t st, int blocks, bool ch, int V, int G) {
    return launch_fn_tmpl<KGE_INTERHT>(p, kind, st, blocks, ch, V, G);
}
}  // namespace kge_impl
