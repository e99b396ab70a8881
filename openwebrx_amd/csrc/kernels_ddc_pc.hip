// kernels_ddc_pc.hip -- explicit instantiations of the DDC kernels (ddc_kernels.h) for
// polyphase depths 8, 16; split so the unrolled kernels compile in parallel.
#include "ddc_kernels.h"

namespace owrx {
OWRX_DDC_INSTANTIATE(, 8)
OWRX_DDC_INSTANTIATE(, 16)
}  // namespace owrx
