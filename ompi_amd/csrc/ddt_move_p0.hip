// ddt_move_p0.hip -- the move kernel instantiated for pack, affine and fragment items only
// (ddt_move.hip.h); one of four translation units the build compiles in parallel.
#include "ddt_move.hip.h"

namespace ddt {
DDT_MOVE_INSTANCE(0, false, p0)
DDT_DENSE_INSTANCE(0, p0)
DDT_SLOT_INSTANCE(0, p0)
}  // namespace ddt
