// tuning.hip — launch variants for A/B timing (scripts/kbench.py).
//
// Compiled only into libzseek_amd/lib/libzseek_tune.so (-DZSK_TUNING); the
// product library libzseek.so carries the production kernels alone.  A
// variant is a route, a subset of the two-phase decoder's stages, or a
// diagnostic build of one kernel (wrong output, timing only).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

#include "zsk_internal.h"

namespace zsk {

namespace {
std::mutex g_mu;
SplitScratch g_s;

int staged(int stages, int route, int tune, const FrameDesc *d_desc, uint32_t nframes,
           const uint8_t *d_comp, uint8_t *d_out, int32_t *d_status, hipStream_t stream)
{
    std::lock_guard<std::mutex> g(g_mu);
    uint64_t want = (uint64_t)nframes * slots_of(65536 + 64);
    if (want > (512ull << 20))
        want = 512ull << 20;
    if (g_s.total && *g_s.total > want)
        want = *g_s.total;
    if (split_scratch_reserve(&g_s, nframes, want, stream) != 0)
        return -1;
    return launch_lz4_split(d_desc, nframes, d_comp, d_out, d_status, nullptr, stream, &g_s, route,
                            stages, tune);
}
// Parse / execute overlap (verdict r04 item 4): the plan on the caller's
// stream, then K frame chunks: chunk c's lean parse on a second stream, its
// execute on the caller's stream after it -- chunk c + 1 parses while chunk c
// executes.  (Every frame takes the lean parse: config 2's route.)
int overlapped(uint32_t K, const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp, uint8_t *d_out,
               int32_t *d_status, hipStream_t stream)
{
    std::lock_guard<std::mutex> g(g_mu);
    static hipStream_t ps = nullptr;
    static hipEvent_t ev[17];
    if (!ps) {
        if (hipStreamCreateWithFlags(&ps, hipStreamNonBlocking) != hipSuccess)
            return -1;
        for (auto &e : ev)
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
                return -1;
    }
    if (K < 1 || K > 16)
        return -1;
    uint64_t want = (uint64_t)nframes * slots_of(65536 + 64);
    if (want > (512ull << 20))
        want = 512ull << 20;
    if (g_s.total && *g_s.total > want)
        want = *g_s.total;
    if (split_scratch_reserve(&g_s, nframes, want, stream) != 0)
        return -1;
    if (launch_lz4_split(d_desc, nframes, d_comp, d_out, d_status, nullptr, stream, &g_s, ROUTE_AUTO, 1, 0) != 0)
        return -1;
    if (hipEventRecord(ev[16], stream) != hipSuccess || hipStreamWaitEvent(ps, ev[16], 0) != hipSuccess)
        return -1;
    for (uint32_t c = 0; c < K; c++) {
        const uint32_t f0 = (uint32_t)((uint64_t)nframes * c / K), f1 = (uint32_t)((uint64_t)nframes * (c + 1) / K);
        if (launch_lz4_lean(d_desc + f0, f1 - f0, d_comp, g_s.rec_base + f0, (uint64_t)g_s.items_cap, g_s.items,
                            g_s.nitems + f0, d_status + f0, nullptr, ps, 0xFFFFFFFFu, 0, 0) != 0)
            return -1;
        if (hipEventRecord(ev[c], ps) != hipSuccess || hipStreamWaitEvent(stream, ev[c], 0) != hipSuccess)
            return -1;
        if (launch_seq_exec(d_desc + f0, f1 - f0, d_comp, d_out, g_s.rec_base + f0, g_s.items, g_s.nitems + f0,
                            d_status + f0, stream) != 0)
            return -1;
    }
    return 0;
}
}   // namespace

// variant:
//   0          production (launch_lz4_frames)
//   1..4       routes: wave / lean / scan / chunk for every frame
//   10 + r     plan + parse only (route r)
//   20         execute only, over the items the previous launch left
//   0x1xx      execute diagnostic DIAG = xx alone (seq_exec.hip; 0x110 prints
//              section timers)
//   0x3xx      execute diagnostic version 0x3xx alone (seq_exec.hip: parts of
//              the dependency rounds removed)
//   0x2xx      plan + lean parse with diagnostic bits xx (lz4_lean.hip;
//              0x204 prints sub-step counters)
//   0x50K      plan, then K frame chunks, chunk c + 1's lean parse on a
//              second stream beside chunk c's execute (0x501 = no overlap)
//   0x400      execute alone with round 0 direct (copy_direct); 0x401 the
//              whole decode with it; 0x402 the whole decode, production
//              execute, same scratch (control)
int launch_lz4_frames_variant(int variant, const FrameDesc *d_desc, uint32_t nframes,
                              const uint8_t *d_comp, uint8_t *d_out, int32_t *d_status,
                              hipStream_t stream)
{
    if (nframes == 0)
        return 0;
    if (variant == 0)
        return launch_lz4_frames(d_desc, nframes, d_comp, d_out, d_status, nullptr, stream);
    if (variant >= 1 && variant <= 4)
        return launch_lz4_frames(d_desc, nframes, d_comp, d_out, d_status, nullptr, stream, variant);
    if (variant >= 10 && variant <= 14)
        return staged(3, variant - 10, 0, d_desc, nframes, d_comp, d_out, d_status, stream);
    if (variant == 20)
        return staged(4, ROUTE_AUTO, 0, d_desc, nframes, d_comp, d_out, d_status, stream);
    if ((variant & 0xF00) == 0x100)
        return staged(4, ROUTE_AUTO, (variant & 0x1FF) << 8, d_desc, nframes, d_comp, d_out, d_status,
                      stream);
    if ((variant & 0xF00) == 0x300)   // execute diagnostics DIAG >= 256 (seq_exec.hip)
        return staged(4, ROUTE_AUTO, (variant & 0x3FF) << 8, d_desc, nframes, d_comp, d_out, d_status, stream);
    if ((variant & 0xF00) == 0x200)
        return staged(3, ROUTE_LEAN, variant & 0xFF, d_desc, nframes, d_comp, d_out, d_status, stream);
    if (variant == 0x400)   // execute alone, round 0 direct (seq_exec.hip copy_direct)
        return staged(4, ROUTE_AUTO, 0x400 << 8, d_desc, nframes, d_comp, d_out, d_status, stream);
    if (variant == 0x401)   // the whole decode with it
        return staged(15, ROUTE_AUTO, 0x400 << 8, d_desc, nframes, d_comp, d_out, d_status, stream);
    if (variant == 0x402)   // the whole decode through the same scratch, production execute (control)
        return staged(15, ROUTE_AUTO, 0, d_desc, nframes, d_comp, d_out, d_status, stream);
    if ((variant & 0xF00) == 0x700)   // execute alone, round-6 candidates (seq_exec.hip 0x7xx)
        return staged(4, ROUTE_AUTO, (variant & 0xFFF) << 8, d_desc, nframes, d_comp, d_out, d_status, stream);
    if ((variant & 0xF00) == 0x800)   // execute alone, traffic split (seq_exec_tune.hip 0x81x)
        return staged(4, ROUTE_AUTO, (variant & 0xFFF) << 8, d_desc, nframes, d_comp, d_out, d_status, stream);
    if ((variant & 0xF00) == 0x600)   // execute alone at W = variant & 0xF waves per SIMD (LDS padding)
        return staged(4, ROUTE_AUTO, (variant & 0xFFF) << 8, d_desc, nframes, d_comp, d_out, d_status, stream);
    if ((variant & 0xF00) == 0x500)   // plan, then K = variant & 0xFF chunks: parse beside the execute
        return overlapped((uint32_t)(variant & 0xFF), d_desc, nframes, d_comp, d_out, d_status, stream);
    return -1;
}

}   // namespace zsk
