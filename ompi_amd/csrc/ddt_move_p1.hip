// ddt_move_p1.hip -- the move kernel instantiated for pack, index-list paths included
// (ddt_move.hip.h); one of four translation units the build compiles in parallel.
#include "ddt_move.hip.h"

namespace ddt {
DDT_MOVE_INSTANCE(0, true, p1)
}  // namespace ddt
