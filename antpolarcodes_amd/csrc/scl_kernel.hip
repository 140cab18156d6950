// scl_kernel.hip -- batched SCL decoding (placeholder until the list kernel lands).
#include "kernels.hpp"

namespace pcg {
int scl_layout(uint32_t, uint32_t, uint32_t* w, uint32_t* l, uint64_t* s)
{
    *w = 0; *l = 0; *s = 0;
    return -4;
}
uint64_t scl_scratch_frames(uint64_t F) { return F; }
int launch_scl(const KernelArgs&, hipStream_t) { return -4; }
} // namespace pcg
