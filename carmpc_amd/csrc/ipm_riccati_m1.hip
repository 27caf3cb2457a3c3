// ipm_riccati_m1.hip -- instantiations of the grouped Riccati kernel for the iteration launch of the pipeline.
#include "ipm_riccati_kernel.h"

namespace carmpc {
namespace ric {
RIC_INST(, false, 1)
RIC_INST_ONESEG(, 1)
}  // namespace ric
}  // namespace carmpc
RIC_TIMING_READER(m1)
