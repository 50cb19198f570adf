// Tile kernels for W = 256, C = 1, with the in-lane spectral features (see tile.hip.h). One TU per
// (W, C, spectral) so the heavily unrolled instantiations build in parallel.
#define MHF_TILE_IMPL
#include "tile.hip.h"

MHF_DEFINE_TILE_LAUNCH(256, 1, 1)
