// ipm_riccati_m0.hip -- instantiations of the grouped Riccati kernel for the single kernel (complete algorithm; small batches, caller-owned instance lists, the pipeline's retry launch).
#include "ipm_riccati_kernel.h"

namespace carmpc {
namespace ric {
RIC_INST(, false, 0)
RIC_INST_ONESEG(, 0)
}  // namespace ric
}  // namespace carmpc
RIC_TIMING_READER(m0)
