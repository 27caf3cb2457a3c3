// ipm_riccati_het.hip -- instantiations of the grouped Riccati kernel for per-instance models (carmpc_hetero_*).
#include "ipm_riccati_kernel.h"

namespace carmpc {
namespace ric {
RIC_INST(, true, 0)
}  // namespace ric
}  // namespace carmpc
RIC_TIMING_READER(het)
