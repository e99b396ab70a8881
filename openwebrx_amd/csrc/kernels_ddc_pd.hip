// kernels_ddc_pd.hip -- explicit instantiations of the DDC kernels (ddc_kernels.h) for
// polyphase depths 32, 48, 64; split so the unrolled kernels compile in parallel.
#include "ddc_kernels.h"

namespace owrx {
OWRX_DDC_INSTANTIATE(, 32)
OWRX_DDC_INSTANTIATE(, 48)
OWRX_DDC_INSTANTIATE(, 64)
}  // namespace owrx
