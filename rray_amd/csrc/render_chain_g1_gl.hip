// render_chain_g1_gl.hip — reflection-chain kernels (render_levels.inc chain_kernel) for G = 1 (scenes with groups),
// culls read from global memory.  A translation unit of their own: build.py compiles these without machine LICM, which otherwise
// hoists constant materialisations (OCML pow's coefficients) out of the chain loop and spills them.
#include <cstdlib>

#include "device_core.inc"
#include "kernels.hpp"
#include "wavefront.hpp"

namespace rr {
#include "render_common.inc"
#include "render_levels.inc"

template void launch_chain_t<1, false>(const DevScene&, const LevelArgs&, hipStream_t, KernelProf*, bool);
}  // namespace rr
