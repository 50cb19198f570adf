// Tile kernels for W = 128, C = 3, moments only (see tile.hip.h). One TU per
// (W, C, spectral) so the heavily unrolled instantiations build in parallel.
#define MHF_TILE_IMPL
#include "tile.hip.h"

MHF_DEFINE_TILE_LAUNCH(128, 3, 0)
