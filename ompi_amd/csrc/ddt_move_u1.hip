// ddt_move_u1.hip -- the move kernel instantiated for unpack, index-list paths included
// (ddt_move.hip.h); one of four translation units the build compiles in parallel.
#include "ddt_move.hip.h"

namespace ddt {
DDT_MOVE_INSTANCE(1, true, u1)
}  // namespace ddt
