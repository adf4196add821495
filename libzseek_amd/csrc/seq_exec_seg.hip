// seq_exec_seg.hip — the execute kernel's block-route instantiation
// (seq_exec_dev.h, SEG = true: items read job by job) in a translation unit
// of its own (in one module with the production instantiation it cost that
// kernel a VGPR spill).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "seq_exec_dev.h"

namespace zsk {

int launch_seq_exec_seg(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp, uint8_t *d_out,
                        const uint64_t *rec_base, const uint64_t *items, const uint32_t *nitems,
                        const int32_t *d_status, hipStream_t stream, const SplitScratch *blk)
{
    if (nframes == 0)
        return 0;
    hipLaunchKernelGGL((seq_exec_kernel<4096, true>), dim3((nframes + kXW - 1) / kXW), dim3(64 * kXW), 0, stream,
                       d_desc, nframes, d_comp, d_out, rec_base, items, nitems, d_status, nullptr, blk->bfirst,
                       blk->bcount, blk->jobs, blk->jres, 0xFFFFFFFFu, 0u);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}   // namespace zsk
