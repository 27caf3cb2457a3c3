// ipm_riccati_m2.hip -- instantiations of the grouped Riccati kernel for the polish launch of the pipeline.
#include "ipm_riccati_kernel.h"

namespace carmpc {
namespace ric {
RIC_INST(, false, 2)
RIC_INST_ONESEG(, 2)
}  // namespace ric
}  // namespace carmpc
RIC_TIMING_READER(m2)
