// so_run.h — the persistent P-frame run's host/device interface, shared by so_me.hip (the
// kernels and launchers) and so_capi.hip (the C-ABI entry points), so both translation units
// see one definition of the kernel-argument structs.
#pragma once
#include "so_common.h"

namespace so {

constexpr int kRunMax = 32;   // frames per persistent launch (kernel-argument table)

// Outputs of one frame (pointers relative to block row by0 of the launch).
struct PFrameOut {
    uint8_t* split;
    int16_t* mv;
    int16_t* qtc;
    int32_t* tokens;
    int32_t* mae;
    uint8_t* recon;
    int32_t* sse;
    int32_t* qpmap;   // two-pass runs: the per-block QP used (so_encode_p_run_2pass); else null
};

// A rank's stripe of a frame shared across GPUs (so_encode_p_run_stripe): block rows [by0, by1)
// of every frame, the reconstruction planes in uncached memory addressed by "virtual" full-frame
// bases (row y at base + y * W; the allocation holds rows [16 * by0 - 16, 16 * by1 + 32)), and
// the hand-off with the neighbouring ranks:
//   * a tile in the stripe's first (last) tile row also stores its top (bottom) 16 recon rows
//     into the up (down) neighbour's plane of the frame (system-scope write-through stores over
//     xGMI) and, once every storing wave has drained, sets that neighbour's flag
//     dn_flags[gf * tiles_x + tx] (up_flags[...]) to `epoch` (system scope);
//   * a tile in the first (last) tile row additionally waits for my_up (my_dn) flags
//     [(gf - 1) * tiles_x + tx - 1 .. tx + 1] == epoch: the rows its window reads from the
//     neighbour's stripe.  Epochs (one per GOP) mean the flag arrays are never reset, so a fast
//     neighbour can never have its flag erased by a slow rank's reset.
// peer planes of global frame gf: peer_*0 + gf * stride.  All-null peers / flags: one GPU.
struct PRunStripe {
    int by0, by1;
    uint8_t* peer_up0;
    uint8_t* peer_dn0;
    long long stride;
    const uint32_t* my_up_flags;
    const uint32_t* my_dn_flags;
    uint32_t* peer_up_flags;   // the up neighbour's my_dn_flags, mapped here
    uint32_t* peer_dn_flags;   // the down neighbour's my_up_flags
    uint32_t epoch;
    int gbase;                 // global frame index (frame pipeline: slot) of the launch's first frame
    // frame pipeline (kRunFPipe): frame j of this rank's run (its slot) predicts from the
    // reconstruction a ring neighbour pushed into land0 + j * stride, with my_dn_flags
    // [j * ntiles + tile] == epoch once that tile arrived; frame j's tiles are pushed per the
    // run's push codes (PRunArgs::dep: slot * 2 + (0: peer_dn, 1: peer_up), -1: no push)
    const uint8_t* land0;
    // two-pass runs (kRunTwoPass): pass-1 done flags [f * ntiles + tile] = epoch, pass-1 token
    // counts [f * nb + b] (both in the workspace), the ROI offsets (int32 [nb] or null) and the
    // QP clamp
    uint32_t* p1done;
    int32_t* t1;
    const int32_t* roi;
    int qp_lo, qp_hi;
    int p2lag;   // tile rows between a row's pass-1 and pass-2 tasks in the queue (1..ntr)
    int count_ops;   // count the searches' SAD byte operations (SO_OPT_COUNT_SAD_OPS)
    int lose_task;   // one GPU: task + 1 whose done flag is never set (SO_OPT_TEST_LOSE_FLAG), 0: none
};

size_t p_run_workspace_words(int H, int W);
int p_run_capacity(int vbs, int mode = -1);
bool p_run_2pass_fused_ok(int H, int W);
int32_t* p_run_t1_region(uint32_t* ws, int H, int W);
// vbs / lam: VBSEnable (the block + sub-block search and the RD split inside the run)
int p_run_launch(const uint8_t* const* curs, int nframes, const uint8_t* ref0, int H, int W, int qp_rd,
                 const int32_t* qp_row, int vbs, double lam, const PFrameOut* outs, uint32_t* ws, hipStream_t st);
int p_runs_launch(const uint8_t* const* curs, int nframes, const uint8_t* const* refs, const int* deps, int conc,
                  int H, int W, int qp_rd, const int32_t* qp_row, int vbs, double lam, const PFrameOut* outs,
                  uint32_t* ws, hipStream_t st);
int p_run_2pass_launch(const uint8_t* const* curs, int nframes, const uint8_t* ref0, int H, int W, int qp_rd,
                       const int32_t* qp_row, const int32_t* roi, int qp_lo, int qp_hi, const PFrameOut* outs,
                       uint32_t* ws, hipStream_t st);
int p_run_stripe_launch(const uint8_t* const* curs, int nframes, const uint8_t* ref0, int H, int W, int qp_rd,
                        const int32_t* qp_row, const PFrameOut* outs, uint32_t* ws, const PRunStripe& sp, int max_wg,
                        hipStream_t st);
int p_run_fpipe_launch(const uint8_t* const* curs, int nframes, int H, int W, int qp_rd, const int32_t* qp_row,
                       int vbs, double lam, const PFrameOut* outs, uint32_t* ws, const PRunStripe& sp, int max_wg,
                       hipStream_t st, const int* push);
int p_run_fpipe_2pass_launch(const uint8_t* const* curs, int nframes, int H, int W, int qp_rd, const int32_t* qp_row,
                             const PFrameOut* outs, uint32_t* ws, const PRunStripe& sp, int max_wg, hipStream_t st,
                             const int* push);

}  // namespace so
