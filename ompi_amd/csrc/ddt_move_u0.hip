// ddt_move_u0.hip -- the move kernel instantiated for unpack, affine and fragment items only
// (ddt_move.hip.h); one of four translation units the build compiles in parallel.
#include "ddt_move.hip.h"

namespace ddt {
DDT_MOVE_INSTANCE(1, false, u0)
DDT_DENSE_INSTANCE(1, u0)
DDT_SLOT_INSTANCE(1, u0)
}  // namespace ddt
