// kernels_ddc_pb.hip -- explicit instantiations of the DDC kernels (ddc_kernels.h) for
// polyphase depth 28; split so the unrolled kernels compile in parallel.
#include "ddc_kernels.h"

namespace owrx {
OWRX_DDC_INSTANTIATE(, 28)
}  // namespace owrx
