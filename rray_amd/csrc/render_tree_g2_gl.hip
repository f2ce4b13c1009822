// render_tree_g2_gl.hip — color_at tree kernels of scenes with transparent materials (render_tree.inc tree_kernel)
// for G = 2 (general shapes and CSG), culls read through the caches.  Built like the chain units (no machine LICM: the loop's constants are
// rematerialised rather than hoisted and spilled).
#include <cstdlib>

#include "device_core.inc"
#include "kernels.hpp"
#include "wavefront.hpp"

namespace rr {
#include "render_common.inc"
#include "render_levels.inc"
#include "render_tree.inc"

template void launch_tree_t<2, false>(const DevScene&, const LevelArgs&, hipStream_t, KernelProf*);
}  // namespace rr
