// gol_step_g9.hip -- instantiates the 9-generation-per-pass step kernels
// (one translation unit per pass depth so they compile in parallel).
#include "gol_stencil.h"

namespace gol {

hipError_t launch_step_g9(const StepParams& p, int vec, bool life, bool hash, bool clipped, int ilv, int gx,
                          int gy, hipStream_t st) {
    return dev::launch_gens<9>(p, vec, life, hash, clipped, ilv, gx, gy, st);
}

int blocks_step_g9(int vec, bool life, bool hash, bool clipped, int ilv) {
    return dev::blocks_gens<9>(vec, life, hash, clipped, ilv);
}

}  // namespace gol
