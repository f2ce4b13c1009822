// render_tree_g1_lds.hip — color_at tree kernels of scenes with transparent materials (render_tree.inc tree_kernel)
// for G = 1 (scenes with groups), culls staged in LDS.  Built like the chain units (no machine LICM: the loop's constants are
// rematerialised rather than hoisted and spilled).
#include <cstdlib>

#include "device_core.inc"
#include "kernels.hpp"
#include "wavefront.hpp"

namespace rr {
#include "render_common.inc"
#include "render_levels.inc"
#include "render_tree.inc"

template void launch_tree_t<1, true>(const DevScene&, const LevelArgs&, hipStream_t, KernelProf*);
}  // namespace rr
