// Indexed register-tile kernels for C = 1 (see tile_idx.hip.h).
#include "tile_idx.hip.h"

namespace mhf {
template int launch_tile_idx_c<1, false>(const IdxTileArgs& a, hipStream_t stream);
}  // namespace mhf
