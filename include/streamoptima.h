/*
 * streamoptima.h — C-ABI of libstreamoptima_hip.so, the MI355X (gfx950) per-block
 * encode path of a StreamOptima-compatible block video encoder.
 *
 * The reference (Suyashagarw/StreamOptima) is pure Python and has no FFI: its drop-in
 * boundary is the Y_Video_codec / decoder Python API.  Each entry point below replaces
 * the reference functions cited next to it; the Python facade in streamoptima_amd/
 * (Encoder.py, decoder.py) keeps the reference's method names and calls these through
 * ctypes (see INTEGRATION.md for the binding).
 *
 * Conventions
 *  - Frames are uint8, row-major, pitch == width, resident in device (HBM) memory; every
 *    frame buffer must be readable for 16 bytes past its last pixel.
 *  - H and W are the encoded frame size and must be multiples of bs (the reference's
 *    pad_hw, Encoder.py:140-155, is applied by the caller; see DESIGN.md for 1080p).
 *  - Blocks are numbered in raster order, nb = (H/bs) * (W/bs).
 *  - All pointers except `refs` (a HOST array of device pointers) are device pointers
 *    allocated by the caller (PyTorch tensors in the facade).  The library never
 *    allocates device memory; all calls are asynchronous on `stream` (a hipStream_t).
 *  - Return 0 (SO_OK) on success, SO_E_* (< 0) for bad arguments, or a positive
 *    hipError_t.  so_last_error() returns a thread-local message for the last failure.
 *  - No C++ exception crosses this boundary.
 *
 * Canonical output layout (shared with tests/golden and the CPU oracle):
 *   split[nb]            uint8   1 = variable-block-size split (4 sub-blocks, Z order)
 *   inter mv[nb][4][3]   int16   (dx, dy, ref) per sub-block; unsplit => entry 0 only
 *   intra mv[nb][4]      int16   dx per sub-block (-1 for blocks at x == 0)
 *   qtc[nb][bs*bs]       int16   quantised coefficients; split => 4 x (bs/2)^2 Z order
 *   tokens[nb]           int32   len(entropy_encoder_block(...)) summed over sub-blocks
 *   mae_num[nb]          int32   block MAE * bs*bs (an integer SAD), -1 = inf
 */
#ifndef STREAMOPTIMA_H
#define STREAMOPTIMA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SO_OK 0
#define SO_E_INVALID (-1)      /* bad argument (message in so_last_error) */
#define SO_E_UNSUPPORTED (-2)  /* valid in the reference but not built for gfx950 yet */
#define SO_MAX_REF 4           /* nRefFrames supported by the kernels */
#define SO_ABI_VERSION 1

/* library identification / diagnostics */
int so_abi_version(void);
const char* so_last_error(void);

/*
 * Full-search integer-pel motion estimation for every bs x bs block of `cur`.
 * Replaces find_best_match + compute_mae + is_better_mv (Encoder.py:678-717, 314-315,
 * 771-773) as called from inter_prediction (Encoder.py:505-562).
 *   refs[nref]   host array of device pointers to H x W reference frames
 *   sr           search range (dx, dy in [-sr, sr]); candidate valid iff
 *                0 <= x+dx < W-bs and 0 <= y+dy < H-bs (strict, like the reference)
 *   out_best     int32 [nb][4]: (dx, dy, ref, sad); sad = -1 if no candidate is valid
 *   out_sub      optional int32 [nb][4][4]: the same for the four (bs/2) sub-blocks of
 *                every block (VBSEnable, Encoder.py:512-544); NULL to skip
 */
int so_me_full_search(const uint8_t* cur, const uint8_t* const* refs, int nref, int H,
                      int W, int bs, int sr, int32_t* out_best, int32_t* out_sub,
                      void* stream);

/*
 * Residual, DCT, quantisation, token count, VBS rate-distortion split decision,
 * dequantisation, IDCT and reconstruction for every block of a P-frame.
 * Replaces calculate_inter_frame_residual (Encoder.py:432-460), apply_2d_dct (:779),
 * quantize_TC (:787), entropy_encoder_block's length (:1086), calculate_RD_cost (:1133)
 * and the split decision (:564-578), the per-block loop of complete_inter_flow
 * (:1665-1697) and reconstruct_frame / reconstruct_block (:824-932).
 *   best/sub     outputs of so_me_full_search (sub may be NULL when vbs == 0)
 *   qp_rd        QP in effect during inter_prediction (used for the RD decision)
 *   qp_row       device int32 [H/bs] per-row QP (rate control), or NULL => qp_rd
 *   lam          lambda of calculate_RD_cost
 *   out_recon    H x W uint8 reconstruction (may not alias any ref)
 *   out_sse      optional int32 [nb]: per-block sum of (cur - recon)^2, for the PSNR of
 *                calculate_metrics (Encoder.py:934) without a separate frame pass; NULL to skip
 */
int so_inter_tq_recon(const uint8_t* cur, const uint8_t* const* refs, int nref, int H,
                      int W, int bs, const int32_t* best, const int32_t* sub, int qp_rd,
                      const int32_t* qp_row, int vbs, double lam, uint8_t* out_split,
                      int16_t* out_mv, int16_t* out_qtc, int32_t* out_tokens,
                      int32_t* out_mae_num, uint8_t* out_recon, int32_t* out_sse, void* stream);

/* int32 elements of scratch so_encode_p_frame needs: nb*4 (+ nb*16 with vbs), + 49,152 for the
 * segment records of the speculated fast-ME predictor chain (so_encode_p_rows_ex) */
size_t so_p_frame_scratch_elems(int H, int W, int bs, int vbs);

/*
 * One P-frame of complete_inter_flow (Encoder.py:1644-1709): so_me_full_search then
 * so_inter_tq_recon, with `scratch` (device int32, so_p_frame_scratch_elems) between.
 */
int so_encode_p_frame(const uint8_t* cur, const uint8_t* const* refs, int nref, int H,
                      int W, int bs, int sr, int qp_rd, const int32_t* qp_row, int vbs,
                      double lam, uint8_t* out_split, int16_t* out_mv, int16_t* out_qtc,
                      int32_t* out_tokens, int32_t* out_mae_num, uint8_t* out_recon,
                      int32_t* out_sse, int32_t* scratch, void* stream);

/*
 * Stripe variant of so_encode_p_frame for multi-GPU sharding: encodes only
 * the block rows [by0, by1) of the frame.  cur, refs and out_recon are still the FULL
 * H x W planes (the search reads the whole reference; only the stripe's pixel rows of
 * out_recon are written).  Symbol outputs (split, mv, qtc, tokens, mae_num, sse) and the
 * scratch are STRIPE-LOCAL: block (bx, by) is record (by - by0) * (W/bs) + bx.  qp_row is
 * the full-frame [H/bs] array.  Concatenating the stripes of by0 = 0 .. H/bs in order
 * reproduces so_encode_p_frame exactly.  so_p_frame_scratch_elems(H, W, ...) suffices.
 */
int so_encode_p_rows(const uint8_t* cur, const uint8_t* const* refs, int nref, int H, int W,
                     int bs, int sr, int by0, int by1, int qp_rd, const int32_t* qp_row,
                     int vbs, double lam, uint8_t* out_split, int16_t* out_mv,
                     int16_t* out_qtc, int32_t* out_tokens, int32_t* out_mae_num,
                     uint8_t* out_recon, int32_t* out_sse, int32_t* scratch, void* stream);

/*
 * Process-wide options of the library (explicit calls, not environment variables; the A/B
 * knobs of the development tools exist only in -DSO_AB builds).  Set them before enqueueing
 * the work they affect; they are read on the host when a call enqueues its launches.
 *   SO_OPT_RUN_2PASS_FUSED   so_encode_p_run_2pass runs both passes of every frame in ONE
 *                            persistent launch (1, default: measured faster, DESIGN.md section 5;
 *                            frames of three or more 32-row tile rows) or as the per-frame kernel
 *                            sequence (0)
 *   SO_OPT_FASTME_SERIAL     fast_me under ParallelMode 0: the one-wavefront serial walk of the
 *                            predictor chain (1) instead of the speculated segments (0, default)
 *   SO_OPT_FASTME_SEGMENT    blocks per speculated segment (default 32, >= 1)
 *   SO_OPT_FASTME_WARMUP     blocks a segment's guess runs ahead of it (default 32, >= 0)
 *   SO_OPT_COUNT_SAD_OPS     the one-GPU persistent runs (so_encode_p_run / _runs) count their
 *                            searches' SAD byte operations into workspace words 66..67 (1; default
 *                            0: a separate test-hook kernel instantiation runs while it is set,
 *                            so the product kernels carry no counting code)
 *   SO_OPT_RUN_ZERO_SKIP     the one-GPU plain run (so_encode_p_run / _runs, VBS off) launches the
 *                            instantiation whose waves skip the IDCT when all their blocks
 *                            quantised to zero (1; exact either way: an all-zero block's inverse
 *                            is zero).  Faster where most blocks are zero (flat content), a
 *                            little slower elsewhere; default 0.  The Python engine sets it per
 *                            run from the previous run's share of all-zero blocks.
 * so_set_option returns SO_E_INVALID for an unknown option or a value out of range.
 */
#define SO_OPT_RUN_2PASS_FUSED 1
#define SO_OPT_FASTME_SERIAL 2
#define SO_OPT_FASTME_SEGMENT 3
#define SO_OPT_FASTME_WARMUP 4
#define SO_OPT_COUNT_SAD_OPS 5
/* TEST ONLY -- never set it around work whose output is used.  SO_OPT_TEST_LOSE_FLAG = k > 0:
 * the next one-GPU run never sets the done flag of its task k - 1, so the tiles that wait on it
 * time out (50 ms each) and record themselves, and that run's symbols are WRONG (the wait
 * diagnostics' test, tests/test_gpu_waits.py).  It is read when a run is enqueued, so a run
 * captured into a graph would stay broken on every replay: a one-GPU run enqueued on a
 * capturing stream while it is set fails with SO_E_INVALID.  Both this option and
 * SO_OPT_COUNT_SAD_OPS select a separate test-hook instantiation of the one-GPU run kernel; the
 * product kernels carry neither hook. */
#define SO_OPT_TEST_LOSE_FLAG 6
#define SO_OPT_RUN_ZERO_SKIP 7
int so_set_option(int option, int value);
int so_get_option(int option);

/*
 * A run of consecutive P-frames (the GOP loop's P-frames between two I-frames,
 * Encoder.py:1839-1867 with nRefFrames 1): frame i predicts from frame i-1's
 * reconstruction (out_recon[i-1]), frame 0 from ref0.  Output is identical to
 * so_encode_p_frame called per frame.  Covers bs 16 / sr 16 with W a multiple of 128 (whole
 * cache lines per tile row); anything else is SO_E_UNSUPPORTED (call so_encode_p_frame per
 * frame).  vbs / lam: VBSEnable and calculate_RD_cost's lambda (Encoder.py:512-578,
 * :1133-1158) -- the block and sub-block search and the RD split run inside the launch
 * (vbs 0: lam unused).
 *
 * One persistent launch per 32 frames: workgroups take (frame, tile) tasks in frame-major
 * raster order, and a tile of frame i starts once the 3x3 tiles of frame i-1 its +-16 px
 * window reads are done (device-scope flags in `workspace`; reconstructions are
 * stored write-through), so consecutive frames overlap on the device with no host
 * round trip.  curs / out_* are host arrays of nframes device pointers; out_sse may be
 * NULL.  workspace: caller-owned uint32 [so_p_run_workspace_elems(H, W)], ZEROED ONCE by the
 * caller before its first use and then only passed back: each launch leaves its counters
 * at 0 and its epoch in the workspace (done flags are compared with the launch's epoch, so
 * nothing is reset between launches).  One workspace serves one stream at a time.  Word 32
 * (SO_P_RUN_TIMEOUT_WORD) is the timeout count: the caller reads it after the run (or after a
 * whole GOP of runs) and clears it (with words 33..35 and the record at 96..127).
 * Nonzero means a dependency wait polled for 50 ms (2 s for another rank's flags; intervals in
 * which the waiting wave was descheduled are not counted) and the run's symbols may be wrong;
 * the facade raises with the record of the first such wait (Engine.check_run).  Consumers poll
 * the flags and then take an agent-scope acquire before reading the reference rows.
 */
#define SO_P_RUN_TIMEOUT_WORD 32
/* Word 64: the number of blocks whose exact SEA search took the dense fallback (more than 192
 * candidates survived the 4x4-cell bound: flat or noise-like content), summed over launches
 * like the timeout count until the caller clears it (a content statistic, not an error). */
#define SO_P_RUN_FALLBACK_WORD 64
/* Words 66..67 (uint64, little endian; with SO_OPT_COUNT_SAD_OPS set): SAD byte operations the
 * searches executed (every
 * v_sad_u8 / v_sad_hi_u8 lane instruction counts its 4 bytes: byte sums, bounds, survivor and
 * dense SADs), summed like word 64.  The dense-equivalent count of the reference's full scan
 * (Encoder.py:688-715) is (valid candidates) x 256 per P-frame; this is what ran. */
#define SO_P_RUN_SAD_OPS_WORD 66
/* Wait health, accumulated like the timeout count ("Waits"):
 * word 33: waits whose relaxed flag polls kept missing a flag for 1 ms of polling that an
 *          atomic read then found set (the wait completes with atomic reads; not an error);
 * word 34: poll intervals longer than 1 ms (the waiting wave was descheduled: compute-queue
 *          preemption), excluded from the wait's bound (not an error). */
#define SO_P_RUN_STALE_WORD 33
#define SO_P_RUN_GAP_WORD 34
/* Words 96..127: the record of the first wait that timed out since word 35 was cleared (all
 * zero: none).  [0] magic 0x534F0001, [1] task, [2] frame (in the launch), [3] dep frame,
 * [4] tile, [5] the launch's epoch (local flags), [6] the GOP epoch (another rank's flags),
 * [7] mode | vbs << 4 | pass << 8 | escalated << 12, [8] lanes waited on (bit l), [9] lanes
 * polling another rank's flags, [10] polling time (100 MHz ticks, gaps excluded), [11] wall
 * ticks, [12] longest poll gap, [13] polls, [14] ticks from the timeout until every awaited
 * flag read set (0xFFFFFFFF: not within 50 ms more), [15] HW_ID, [16] XCC_ID, [17] blockIdx.x,
 * [18] gridDim.x, [19] lanes whose flag an atomic read found set at the timeout,
 * [20 + l] the last value lane l read (l < 12). */
#define SO_P_RUN_DIAG_WORD 96
#define SO_P_RUN_DIAG_MAGIC 0x534F0001u
size_t so_p_run_workspace_elems(int H, int W);
/* The workgroups the persistent run kernel keeps resident on the calling thread's current
 * device (CUs x workgroups per CU; vbs: the VBSEnable kernel): the grid of an uncapped launch.
 * Several ranks' runs sharing ONE device (in-process tests, time-shared rehearsals) must keep
 * the sum of their grids (max_wg of the stripe / frame-pipeline entry points) within it: a
 * launch that cannot become resident would leave the others waiting on its tasks (DESIGN.md
 * section 6, "Forward progress").  SO_E_INVALID if the device query fails. */
int so_p_run_resident_workgroups(int vbs);
/* The same for ONE run kind: mode 0 the one-GPU run (so_encode_p_run / _runs), 1 the stripe
 * run, 2 the frame pipeline, 3 the fused two-pass run, 4 the two-pass frame pipeline (vbs: modes
 * 0 and 2).  so_p_run_resident_workgroups(vbs) is the smallest of these, so a claim sized by it
 * fits whichever kernel a rank launches.  SO_E_INVALID for another mode or a failed query. */
int so_p_run_mode_resident_workgroups(int mode, int vbs);
int so_encode_p_run(const uint8_t* const* curs, int nframes, const uint8_t* ref0, int H, int W,
                    int bs, int sr, int qp_rd, const int32_t* qp_row, int vbs, double lam,
                    uint8_t* const* out_split,
                    int16_t* const* out_mv, int16_t* const* out_qtc, int32_t* const* out_tokens,
                    int32_t* const* out_mae_num, uint8_t* const* out_recon, int32_t* const* out_sse,
                    uint32_t* workspace, void* stream);

/*
 * A run of P-frames with two-pass rate control (build extension, RCFlag 3)
 * in one call: per frame, pass 1 at the rate-control row QP (qp_row, or qp_rd)
 * gives each block's token count t, the per-block QP is clamp(row QP + delta + roi, qp_lo,
 * qp_hi) with delta = [t n >= 2m] + [t n >= 4m] - [2 t n < m] - [4 t n < m] (m = the block
 * row's pass-1 token sum over its n blocks; so_qp_map's rule), and pass 2 re-runs the
 * transforms at those QPs on pass 1's motion vectors.  Identical to the per-frame sequence
 * so_encode_p_rows_ex (pass 1) + so_qp_map + so_encode_p_rows_ex(SO_REUSE_ME) (pass 2);
 * out_qp_map[i] (int32 [nb]) receives frame i's QPs.  roi: int32 [nb] offsets or NULL.  By
 * default both passes run in ONE persistent launch (each task the pass 2 of one tile, then the
 * pass 1 of the tile tiles_x + 1 positions later; a pass 2 waits for its tile row's pass 1);
 * with so_set_option(SO_OPT_RUN_2PASS_FUSED, 0), or for frames of fewer than three 32-row tile
 * rows, the library enqueues the per-frame kernel sequence itself instead (pass 1 tokens-only,
 * pass 2 with the QP map; the ME records kept in the workspace).  Frame i predicts from frame i-1's
 * pass-2 reconstruction, frame 0 from ref0.  Same coverage and workspace as so_encode_p_run
 * (W <= 8192).
 */
/*
 * 1 when so_encode_p_run_2pass runs an H x W frame (bs 16) in the one persistent launch (the
 * option SO_OPT_RUN_2PASS_FUSED is on and the frame has three 32-row tile rows or more, which
 * the merged schedule's deadlock-freedom needs), 0 when it enqueues the per-frame sequence.
 */
int so_p_run_2pass_fused(int H, int W);

int so_encode_p_run_2pass(const uint8_t* const* curs, int nframes, const uint8_t* ref0, int H, int W,
                          int bs, int sr, int qp_rd, const int32_t* qp_row, const int32_t* roi,
                          int qp_lo, int qp_hi, uint8_t* const* out_split, int16_t* const* out_mv,
                          int16_t* const* out_qtc, int32_t* const* out_tokens,
                          int32_t* const* out_mae_num, uint8_t* const* out_recon,
                          int32_t* const* out_sse, int32_t* const* out_qp_map, uint32_t* workspace,
                          void* stream);

/*
 * Several independent runs of P-frames in ONE persistent launch (the P-frames of several
 * GOPs, or of the runs between a GOP's I-frames): frame i predicts from out_recon[j] when
 * ref_frame[i] = j (j < i, a frame of this list: its tiles are waited for inside the launch
 * as in so_encode_p_run) and from refs[i] when ref_frame[i] = -1 (a plane complete before
 * the call, e.g. an I-frame's reconstruction).  Frames are taken in list order, so
 * interleaving the runs (A1 B1 A2 B2 ...) keeps the tiles of one frame of every run in flight
 * at once: where one frame has fewer tiles than the GPU's resident workgroups (1080p), the
 * runs fill the GPU that one run's frame-to-frame dependency leaves idle.  Each run's
 * output is identical to so_encode_p_run of that run alone (the reference's loop,
 * Encoder.py:1839-1867, per GOP).  refs: host array of nframes device pointers (entries with
 * ref_frame >= 0 are ignored); ref_frame: host int32[nframes]; the rest as so_encode_p_run.
 */
int so_encode_p_runs(const uint8_t* const* curs, int nframes, const uint8_t* const* refs,
                     const int32_t* ref_frame, int H, int W, int bs, int sr, int qp_rd,
                     const int32_t* qp_row, int vbs, double lam, uint8_t* const* out_split,
                     int16_t* const* out_mv,
                     int16_t* const* out_qtc, int32_t* const* out_tokens, int32_t* const* out_mae_num,
                     uint8_t* const* out_recon, int32_t* const* out_sse, uint32_t* workspace,
                     void* stream);

/*
 * ONE GOP across the GPUs of a node (BASELINE configs[3]): rank r encodes the block rows
 * [by0, by1) of every P-frame of a run with the persistent kernel of so_encode_p_run, and the
 * stripes hand their boundary rows to each other inside the launch -- the reference's frame
 * dependency (Encoder.py:1864-1867, P(i) searches recon(i-1)) extended across GPUs:
 *   * each rank's reconstruction planes live in UNCACHED device memory (so_alloc_uncached),
 *     addressed by "virtual" full-frame bases (row y of frame gf at base_gf + y * W; the
 *     allocation holds rows [16 by0 - 16, 16 by1 + 32));
 *   * a tile of the stripe's first (last) tile row also stores its top (bottom) 16 rows into
 *     the up (down) neighbour's plane of the frame -- peer memory mapped with so_ipc_open,
 *     reached over xGMI -- with system-scope write-through stores and, once they have drained,
 *     sets the neighbour's flag [gf * tiles_x + tx] (tiles_x = W / 128) to `epoch`;
 *   * a first- (last-) row tile waits, besides its own 3x3 tiles of the frame before, for
 *     my_up_flags (my_dn_flags) [(gf - 1) * tiles_x + tx - 1 .. tx + 1] == epoch.
 * curs: the frames (full H x W planes, only the stripe rows are read); out_recon[i]: virtual
 * bases of the stripe's planes; ref0: the virtual base of frame gbase - 1; symbol outputs are
 * stripe-local as in so_encode_p_rows.  peer_up0 / peer_dn0: the neighbours' virtual bases
 * of frame 0 as mapped here (frame gf at + gf * stride); any of the four neighbour pointers
 * NULL = no neighbour on that side.  epoch: a per-GOP value the flags are compared with
 * (they are never reset).  max_wg > 0 caps the resident grid (ranks sharing one GPU).
 * gbase >= 1 (frame 0 is the GOP's I-frame).
 */
int so_encode_p_run_stripe(const uint8_t* const* curs, int nframes, const uint8_t* ref0, int H, int W,
                           int bs, int sr, int by0, int by1, int qp_rd, const int32_t* qp_row,
                           uint8_t* const* out_split, int16_t* const* out_mv, int16_t* const* out_qtc,
                           int32_t* const* out_tokens, int32_t* const* out_mae_num,
                           uint8_t* const* out_recon, int32_t* const* out_sse, uint32_t* workspace,
                           int gbase, uint8_t* peer_up0, uint8_t* peer_dn0, long long stride,
                           const uint32_t* my_up_flags, const uint32_t* my_dn_flags,
                           uint32_t* peer_up_flags, uint32_t* peer_dn_flags, uint32_t epoch, int max_wg,
                           void* stream);

/* The I-frame's hand-off: rows [16 by0, 16 by0 + 16) of `plane` (a virtual base) to peer_up,
 * rows [16 by1 - 16, 16 by1) to peer_dn (the neighbours' virtual bases of frame gf), then
 * their flags [gf * tiles_x + tx] = epoch.  NULL peer = no neighbour on that side. */
int so_stripe_halo_push(const uint8_t* plane, int H, int W, int by0, int by1, int gf, uint8_t* peer_up,
                        uint8_t* peer_dn, uint32_t* peer_up_flags, uint32_t* peer_dn_flags,
                        uint32_t epoch, void* stream);

/*
 * One GOP across GPUs, consecutive frames on consecutive ranks (the frame pipeline of
 * DESIGN.md §6; north_star "frames within a GOP shard across the GPUs").  Rank g of N encodes
 * the frames k = g + N*j; frame k predicts from frame k-1, encoded by rank g-1 (mod N).  Each
 * rank owns uncached landing planes (so_alloc_uncached; slot j at land0 + j * stride, at least
 * H*W bytes + 16) with one flag word per 128x32 tile (land_flags + j * ntiles, ntiles =
 * (W/128) * ceil(H/32)): slot j holds the reconstruction of frame k-1 for its frame j, flagged
 * tile by tile == epoch as it arrives.  The persistent run of the rank's frames [slot0,
 * slot0 + nframes) waits per tile for the 3x3 arrived tiles of its reference, and stores every
 * tile's reconstruction both into out_recon[i] (local) and, system-scope write-through over
 * xGMI, into the landing plane its push code names before setting that rank's flag to epoch:
 * push_to[i] = 2 * slot + peer puts frame i's reconstruction into slot `slot` of peer_land0
 * (peer 0, flags peer_flags) or of peer2_land0 (peer 1, flags peer2_flags) -- the two ring
 * neighbours, so the ring direction can alternate per block of N frames -- and -1 pushes
 * nothing (the GOP's last frame).  Slots at or past nslots (every rank's slot count) are
 * rejected, as is slot0 + nframes > nslots.  Epochs are never reset (a new GOP uses a new
 * epoch).  vbs / lam as so_encode_p_run.  The symbols are those of so_encode_p_run over the
 * same frames.  so_frame_push sends a finished frame (the I-frame) the same way.  workspace:
 * so_p_run_workspace_elems(H, W), as so_encode_p_run.  max_wg > 0 caps the grid.
 */
int so_encode_p_run_fpipe2(const uint8_t* const* curs, int nframes, int H, int W, int bs, int sr,
                           int qp_rd, const int32_t* qp_row, int vbs, double lam,
                           uint8_t* const* out_split,
                           int16_t* const* out_mv, int16_t* const* out_qtc, int32_t* const* out_tokens,
                           int32_t* const* out_mae_num, uint8_t* const* out_recon,
                           int32_t* const* out_sse, uint32_t* workspace, const uint8_t* land0,
                           const uint32_t* land_flags, int slot0, uint8_t* peer_land0,
                           uint32_t* peer_flags, uint8_t* peer2_land0, uint32_t* peer2_flags,
                           const int32_t* push_to, int nslots, long long stride, uint32_t epoch,
                           int max_wg, void* stream);
/*
 * The frame pipeline with two-pass rate control and ROI (BASELINE configs[4] across GPUs;
 * build extension): each of the rank's frames runs pass 1, the per-block
 * QP map and pass 2 exactly as so_encode_p_run_2pass (roi, qp_lo, qp_hi, out_qp_map as there),
 * tile by tile inside ONE persistent launch (a tile's pass 2 starts once its tile row finished
 * pass 1), and pass 2 pushes the final reconstruction into the next frame's rank as
 * so_encode_p_run_fpipe2 does (same landing planes, flags, push codes, nslots and epochs).
 * A rank owns whole frames, so the row-local QP statistics never cross ranks.  The symbols
 * and QP maps are those of the one-GPU two-pass sequence over the same frames.  A tile row's
 * pass-2 tasks are queued about one grid's worth of tile rows after its pass-1 tasks; p2lag > 0
 * caps that lag (consecutive frames across ranks trail each other by ~lag + 2 tile rows, so
 * more ranks want a shorter one: pipeline.fpipe_p2lag); 0 = no cap.
 */
int so_encode_p_run_fpipe_2pass(const uint8_t* const* curs, int nframes, int H, int W, int bs, int sr,
                                int qp_rd, const int32_t* qp_row, const int32_t* roi, int qp_lo,
                                int qp_hi, uint8_t* const* out_split, int16_t* const* out_mv,
                                int16_t* const* out_qtc, int32_t* const* out_tokens,
                                int32_t* const* out_mae_num, uint8_t* const* out_recon,
                                int32_t* const* out_sse, int32_t* const* out_qp_map, uint32_t* workspace,
                                const uint8_t* land0, const uint32_t* land_flags, int slot0,
                                uint8_t* peer_land0, uint32_t* peer_flags, uint8_t* peer2_land0,
                                uint32_t* peer2_flags, const int32_t* push_to, int nslots, long long stride,
                                uint32_t epoch, int max_wg, int p2lag, void* stream);
int so_frame_push(const uint8_t* plane, int H, int W, uint8_t* peer_plane, uint32_t* peer_flags,
                  uint32_t epoch, void* stream);

/* Device memory the ranks share.  The one exception to "the library never allocates": the
 * landing planes and flags of the cross-GPU hand-off must be uncached
 * (hipExtMallocWithFlags(hipDeviceMallocUncached)), which PyTorch cannot allocate. */
#define SO_IPC_HANDLE_BYTES 64
int so_alloc_uncached(size_t bytes, void** out);
int so_free_device(void* p);
int so_ipc_export(void* p, uint8_t* out_handle);            /* hipIpcGetMemHandle */
int so_ipc_open(const uint8_t* handle, void** out);         /* hipIpcOpenMemHandle */
int so_ipc_close(void* p);
/* stream-ordered copies / fills of such memory (torch cannot wrap it) */
int so_copy_d2d(void* dst, const void* src, size_t bytes, void* stream);
int so_memset_d8(void* dst, int value, size_t bytes, void* stream);

/* int32 elements of scratch so_encode_i_frame / so_intra_recon need: nb*(bs*bs) + nb*8 */
size_t so_i_frame_scratch_elems(int H, int W, int bs);

/*
 * One I-frame of complete_intra_flow, intra_mode 0 (Encoder.py:1582-1642):
 * intra_prediction (:1238-1347, horizontal search intra_find_best_match_horizontal
 * :1010-1045, canvas generalised from the hard-coded 288x352 to H x W), per-block
 * DCT/quant/tokens/VBS-RD, and reconstruct_frame_intra (:1350-1417; unclipped canvas,
 * final astype(uint8) == mod-256 wrap).  out_mv is int16 [nb][4].  out_sse: optional
 * int32 [H] per PIXEL ROW sum of (cur - recon)^2 (the recon is produced row-parallel).
 */
int so_encode_i_frame(const uint8_t* cur, int H, int W, int bs, int sr, int qp_rd,
                      const int32_t* qp_row, int vbs, double lam, uint8_t* out_split,
                      int16_t* out_mv, int16_t* out_qtc, int32_t* out_tokens,
                      int32_t* out_mae_num, uint8_t* out_recon, int32_t* out_sse,
                      int32_t* scratch, void* stream);

/*
 * Stripe variant of so_encode_i_frame: block rows [by0, by1), same conventions as
 * so_encode_p_rows; out_sse is [(by1 - by0) * bs] per pixel row of the stripe.  Intra
 * mode 0 reads only original pixels and its reconstruction is row-local, so stripes need
 * no halo.
 */
int so_encode_i_rows(const uint8_t* cur, int H, int W, int bs, int sr, int by0, int by1,
                     int qp_rd, const int32_t* qp_row, int vbs, double lam, uint8_t* out_split,
                     int16_t* out_mv, int16_t* out_qtc, int32_t* out_tokens,
                     int32_t* out_mae_num, uint8_t* out_recon, int32_t* out_sse,
                     int32_t* scratch, void* stream);

/*
 * ---- ME variants: fast_me and FMEEnable (Encoder.py:388-406, 678-742, 1644-1651) -----------
 *
 * me_mode:
 *   SO_ME_FULL      find_best_match, exhaustive +-sr (the default path above);
 *   SO_ME_FAST      fast_me, serial branch of inter_prediction (:462-585): the 3x3
 *                   neighbourhood of a predictor that is the previous block's mv in raster
 *                   order (starting at (0,0,0)); a serial chain -- ONE wavefront walks the
 *                   frame, so stripes (by0 > 0) are rejected;
 *   SO_ME_FAST_PAR  fast_me under ParallelMode 2 (inter_prediction_parallel :587-676):
 *                   predictor (0,0,0) for every block and nRefFrames 1 (VBS is rejected: the
 *                   reference raises NameError there).
 * fast_me's MAE is the chosen reference INDEX (:742): the ME record's last field is then
 * ref * n^2 (and 0 when no candidate was valid, with mv = the predictor).
 * fme: search the frac frame frac_me_reference_frame(refs) ((2H-1) x (2W-1)) at (2x, 2y) over
 *   half-pel offsets in [-2sr, 2sr]; MVs are in half-pel units.  The library builds the
 *   frame as four phase planes P_ab[i][j] = F[2i+a][2j+b] into the caller's workspace
 *   `fme_planes` (so_fme_workspace_bytes) on every call, with
 *   fme_wrap = 1 when every reference is a uint8 reconstruction (the reference's
 *   `row + np.roll(row, -1)` then wraps mod 256), 0 while the list still holds the float64
 *   all-128 start frame (Encoder.py:1798).
 */
#define SO_ME_FULL 0
#define SO_ME_FAST 1
#define SO_ME_FAST_PAR 2

/* bytes of the FME workspace for nref references: nref * 4 planes of so_fme_plane_stride */
size_t so_fme_plane_stride(int H, int W);
size_t so_fme_workspace_bytes(int H, int W, int nref);

/* The four phase planes of one reference's frac frame (frac_me_reference_frame,
 * Encoder.py:388-403 / decoder.py:468-483) into out_planes (4 x so_fme_plane_stride). */
int so_fme_planes(const uint8_t* ref, int H, int W, int wrap, uint8_t* out_planes, void* stream);

/* so_me_full_search generalised by me_mode / fme (fme_planes: workspace, NULL unless fme). */
int so_me_search_ex(const uint8_t* cur, const uint8_t* const* refs, int nref, int H, int W, int bs,
                    int sr, int me_mode, int fme, int fme_wrap, uint8_t* fme_planes,
                    int32_t* out_best, int32_t* out_sub, void* stream);

/*
 * so_encode_p_rows generalised by me_mode / fme, a per-block QP map and flags; the same
 * outputs and scratch.
 *   qp_map  device int32 [H/bs * W/bs] per-block QP (full-frame, raster) or NULL; it
 *           replaces qp_row / qp_rd for the quantisation and reconstruction of each block
 *           (the VBS RD decision keeps qp_rd, like the reference's); see so_qp_map
 *   flags   SO_REUSE_ME: skip the ME; `scratch` (and fme_planes) still hold the ME records
 *           of a previous call on the same cur / refs / rows (pass 2 of two-pass RC)
 *           SO_TOKENS_ONLY: pass 1 of two-pass RC -- only out_tokens and the ME records in
 *           `scratch` are guaranteed (the fused full-search path skips the rest of the
 *           transform); the other outputs are left for the SO_REUSE_ME pass to write
 */
#define SO_REUSE_ME 1
#define SO_TOKENS_ONLY 2
int so_encode_p_rows_ex(const uint8_t* cur, const uint8_t* const* refs, int nref, int H, int W,
                        int bs, int sr, int by0, int by1, int qp_rd, const int32_t* qp_row,
                        const int32_t* qp_map, int vbs, double lam, int me_mode, int fme,
                        int fme_wrap, uint8_t* fme_planes, int flags, uint8_t* out_split,
                        int16_t* out_mv,
                        int16_t* out_qtc, int32_t* out_tokens, int32_t* out_mae_num,
                        uint8_t* out_recon, int32_t* out_sse, int32_t* scratch, void* stream);

/* Decoder P-frame reconstruction with FMEEnable (decoder.py:97-211 FME branches) and a
 * per-block QP map (NULL: qp_row / qp). */
int so_inter_recon_ex(const uint8_t* const* refs, int nref, int H, int W, int bs, int qp,
                      const int32_t* qp_row, const int32_t* qp_map, int fme, int fme_wrap,
                      uint8_t* fme_planes,
                      const uint8_t* split, const int16_t* mv, const int16_t* qtc,
                      uint8_t* out_recon, void* stream);

/* so_encode_i_rows / so_intra_recon with a per-block QP map (NULL: qp_row / qp_rd). */
int so_encode_i_rows_ex(const uint8_t* cur, int H, int W, int bs, int sr, int by0, int by1,
                        int qp_rd, const int32_t* qp_row, const int32_t* qp_map, int vbs,
                        double lam, uint8_t* out_split, int16_t* out_mv, int16_t* out_qtc,
                        int32_t* out_tokens, int32_t* out_mae_num, uint8_t* out_recon,
                        int32_t* out_sse, int32_t* scratch, void* stream);
int so_intra_recon_ex(int H, int W, int bs, int qp, const int32_t* qp_row, const int32_t* qp_map,
                      const uint8_t* split, const int16_t* mv, const int16_t* qtc,
                      uint8_t* out_recon, int32_t* scratch, void* stream);

/*
 * ROI and two-pass rate control (BASELINE configs[4]; a build extension -- the reference
 * computes per-row stats in complete_*_flow and discards them, Encoder.py:1627-1640,
 * 1696-1707, and has no ROI).  Writes the per-block QP map of block rows [by0, by1):
 *   qp = clamp(base + delta + roi, qp_lo, qp_hi),  base = qp_row[by] or qp_rd,
 *   delta in [-2, 2] from the block's pass-1 token count t against its row's sum m over n
 *   blocks: [t n >= 2m] + [t n >= 4m] - [2 t n < m] - [4 t n < m]  (0 when tokens == NULL).
 *   tokens  device int32 stripe-local pass-1 token counts (so_encode_*_rows out_tokens), or NULL
 *   roi     device int32 [H/bs * W/bs] QP offsets (negative = finer), or NULL
 *   out_qp_map  device int32 [H/bs * W/bs] (rows outside [by0, by1) untouched)
 */
int so_qp_map(const int32_t* tokens, int H, int W, int bs, int by0, int by1, int qp_rd,
              const int32_t* qp_row, const int32_t* roi, int qp_lo, int qp_hi,
              int32_t* out_qp_map, void* stream);

/* Decoder: P-frame reconstruction from symbols (decoder.py:97-211). */
int so_inter_recon(const uint8_t* const* refs, int nref, int H, int W, int bs, int qp,
                   const int32_t* qp_row, const uint8_t* split, const int16_t* mv,
                   const int16_t* qtc, uint8_t* out_recon, void* stream);

/* Decoder: I-frame reconstruction from symbols (decoder.py:330-432, mode 0). */
int so_intra_recon(int H, int W, int bs, int qp, const int32_t* qp_row,
                   const uint8_t* split, const int16_t* mv, const int16_t* qtc,
                   uint8_t* out_recon, int32_t* scratch, void* stream);

/*
 * Batched per-block transforms for the reference's per-block public methods (the drop-in
 * surface): n blocks of N x N doubles (N = 16 or 8), row-major [n][N][N].
 *   inverse 0: out_tc = np.round(DCT-II 2-D)     -- apply_2d_dct (Encoder.py:779-784)
 *              with qp >= 0 also out_q = np.round(TC / Q(N, qp)) -- quantize_TC (:787-789)
 *              and out_tokens[n] = len(entropy_encoder_block(QTC)) (:1086-1131), the
 *              per-block terms of calculate_RD_cost (:1133-1158)
 *   inverse 1: out_tc = np.round(DCT-III 2-D)    -- apply_2d_idct (:810-817), the transform
 *              inside reconstruct_block (:824-827); out_q / out_tokens must be NULL
 * Outputs are device int32 [n][N][N] / [n] (each may be NULL).  Same FP64 operation order as
 * the frame kernels (pocketfft replica, bitwise equal to scipy.fftpack).
 */
int so_block_xform(const double* in, int n, int N, int inverse, int qp, int32_t* out_tc,
                   int32_t* out_q, int32_t* out_tokens, void* stream);

/*
 * Sum of squared differences of two uint8 planes of n pixels, ADDED into *out_sse
 * (device uint64; zero it first).  PSNR per frame (calculate_metrics, Encoder.py:934)
 * is 10*log10(255^2 / (sse / n)) on the host.
 */
int so_sse_u8(const uint8_t* a, const uint8_t* b, int64_t n, uint64_t* out_sse,
              void* stream);

/*
 * out[i] = sum of rows[i][0..len) (int32 -> int64) for i < n: the per-frame SSE of a GOP from
 * the encode kernels' per-block / per-row out_sse arrays (rows: a HOST array of device
 * pointers), one launch.
 */
int so_sum_i32_rows(const int32_t* const* rows, int n, int len, int64_t* out, void* stream);

/*
 * Packed symbol stream: the content of the reference's two text lines per frame
 * (differential_encoder_frame's MVs before differencing, Encoder.py:1419-1520, and
 * entropy_encoder_block's RLE token lists, :1086-1131 / :1522-1542) as zigzag LEB128
 * varints, per block in raster order:  split | mv values | token lists of its (sub-)blocks.
 * Replaces downloading the dense int16 QTC (2 B/px) when symbols leave the GPU
 * (transmit_bitstream, :1544-1580).  Format: so_pack.hip; host decoder: bitstream.unpack_frame.
 *
 * so_pack_bound: the worst-case bytes of a frame of nb blocks (a capacity that never
 *   overflows).
 * so_pack_frames: for frame i (frame_types: a HOST array, 0 = intra, 1 = inter; split / mv /
 *   qtc: device arrays in the canonical symbol layout) writes offs[i][0..nb) = each block's byte offset, offs[i][nb] =
 *   the frame's total, and the stream into out[i][0..total).  Blocks that would pass `cap`
 *   bytes are not written: the caller checks offs[i][nb] <= cap before using out[i].
 *   Stream-ordered, no host synchronisation.
 * so_pack_frames_ex: the same, and totals[i] = offs[i][nb] (totals: nframes uint32, device
 *   memory or page-locked host memory the device can address -- stored at system scope, so a
 *   host that has waited for the stream reads them without a copy; NULL = none).  A host
 *   streaming the packed bytes out learns each frame's length from it without a gather and a
 *   copy per chunk (hoststream.HostStreamEncoder).
 */
size_t so_pack_bound(int nb, int block_size);
int so_pack_frames(int nframes, const int32_t* frame_types, const uint8_t* const* split,
                   const int16_t* const* mv, const int16_t* const* qtc, int nb, int block_size,
                   uint32_t* const* offs, uint8_t* const* out, unsigned long long cap,
                   void* stream);
int so_pack_frames_ex(int nframes, const int32_t* frame_types, const uint8_t* const* split,
                      const int16_t* const* mv, const int16_t* const* qtc, int nb, int block_size,
                      uint32_t* const* offs, uint8_t* const* out, unsigned long long cap,
                      uint32_t* totals, void* stream);

/*
 * The inverse (the decoder side of the packed stream): frame i's bytes packed[i] with the
 * block offsets offs[i][0..nb] so_pack_frames wrote, back to split / mv / qtc in the canonical
 * layout (mv entries past an unsplit block's first are 0).  frame_types: HOST array.
 * Malformed input sets the device int32 *err to 1 + a bad block's index (zero it first).
 */
int so_unpack_frames(int nframes, const int32_t* frame_types, const uint8_t* const* packed,
                     const uint32_t* const* offs, int nb, int block_size, uint8_t* const* split,
                     int16_t* const* mv, int16_t* const* qtc, int32_t* err, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* STREAMOPTIMA_H */
