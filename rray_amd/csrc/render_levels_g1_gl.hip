// render_levels_g1_gl.hip — level kernels for G = 1 (scenes with groups), culls read from global memory.
// One (G, LC) variant per translation unit so the kernel variants compile in parallel (render_levels.inc).
#include <cstdlib>

#include "device_core.inc"
#include "kernels.hpp"
#include "wavefront.hpp"

namespace rr {
#include "render_common.inc"
#include "render_levels.inc"

template void launch_level_t<1, false>(const DevScene&, const LevelArgs&, hipStream_t, KernelProf*);
}  // namespace rr
