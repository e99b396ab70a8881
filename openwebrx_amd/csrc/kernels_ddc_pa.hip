// kernels_ddc_pa.hip -- explicit instantiations of the DDC kernels (ddc_kernels.h) for
// polyphase depth 27; split so the unrolled kernels compile in parallel.
#include "ddc_kernels.h"

namespace owrx {
OWRX_DDC_INSTANTIATE(, 27)
}  // namespace owrx
