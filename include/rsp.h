/*
 * rsp.h -- C ABI of the MI355X range-Doppler engine (pulse compression -> MTD ->
 * zero-velocity suppression -> 2-D CA-CFAR), the drop-in boundary for the hot path
 * of XuZerui2023/Radar-Signal-Process.
 *
 * Plain C linkage, plain pointers and int64 sizes; no C++ or torch types cross it.
 * Each entry point cites the MATLAB interface it replaces (paths relative to the
 * reference root):
 *
 *   rsp_pc_mtd        MTD_Signal = fun_MTD_produce(echoData, params)
 *                     (MTD/fun_MTD_produce.m:12; legacy 1-arg form
 *                      MatlabProcess_xuzerui/fun_MTD_produce.m:3; callers
 *                      MTD/main_produce_dataset_win_xzr_v2.m:136,
 *                      MatlabProcess_xuzerui/main_produce_dataset_win_xzr.m:37-38)
 *   rsp_cfar          [flag, flagV] = executeCFAR(rdm, refR, saveR, TR, mR,
 *                                                 refV, saveV, TV, mV, M0, rFlag)
 *                     (MatlabProcess_xuzerui/CFAR_WangCai/executeCFAR.m:1-2), and with
 *                     nseg > 1 the segmented cfarFlag = fun_CFARflag(...)
 *                     (CFAR_WangCai/main_cfar.m:142-161, a local function there),
 *                     optionally preceded by main_cfar.m:88-91's fun_0v_pressing
 *   rsp_pc_mtd_cfar   the fused chain fun_MTD_produce -> main_cfar's per-window CFAR
 *                     (MTD/main_produce_dataset_win_xzr_v2.m:136 then
 *                      CFAR_WangCai/main_cfar.m:88-93)
 *
 * Conventions
 *   - Every call returns an int status (RSP_OK = 0); the message of the last failure
 *     is rsp_last_error(ctx) (ctx == NULL: the last rsp_create failure).
 *   - Host-buffer entry points (no _dev suffix) are synchronous; the caller owns the
 *     host buffers, the context owns its device buffers (grow-only pool).
 *   - _dev entry points take device pointers and enqueue on `stream` (a hipStream_t,
 *     NULL = the null stream); they return before the work completes.
 *   - One context per host thread and device.  MATLAB calls MEX on one thread.  Contexts
 *     on different threads and devices are independent (kernel launch setup is cached per
 *     device, thread-safely).  _dev calls on one context may use different streams: each
 *     call's stream first waits for the previous call's use of the context's scratch.
 *   - Device layouts are row-major C order: echo [batch][P][R] complex (interleaved
 *     I/Q), RDM [batch][Nd][R_out] float32, flags [batch][Nd][R_out] uint8 0/1, where
 *     Nd = P (Doppler bins) and R_out = params.R_out.
 *   - Host-buffer entry points accept MATLAB column-major (RSP_COLMAJOR: element
 *     (p, r) at r*P + p) or row-major data and convert on the device.
 */
#ifndef RSP_H
#define RSP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RSP_ABI_VERSION 4   /* 2: rsp_set_fused / rsp_chain_check removed, rsp_set_pc_split added;
                               3: rsp_set_host_pipeline;
                               4: rsp_set_flow / rsp_flow_status (round 5's opt-in dataflow launch,
                                  with its RSP_K_FLOW profile slot) removed; rsp_set_range_concat
                                  added; rsp_profile_read_n
                                  takes the arrays' length, rsp_profile_read writes exactly the 4
                                  ABI-3 entries */
#define RSP_MAX_SEG 4
#define RSP_MAX_FIR_TAPS 64

typedef struct rsp_ctx rsp_ctx;

typedef enum {
    RSP_OK = 0,
    RSP_ERR_ARG = 1,          /* bad pointer / enum / size */
    RSP_ERR_SHAPE = 2,        /* P, R, batch inconsistent with the context's params */
    RSP_ERR_UNSUPPORTED = 3,  /* valid in MATLAB but not built here (e.g. odd FFT size) */
    RSP_ERR_CFAR_WINDOW = 4,  /* a CFAR window does not fit: MATLAB raises an index error */
    RSP_ERR_HIP = 5,          /* HIP runtime error (message has the HIP string) */
    RSP_ERR_NOMEM = 6
} rsp_status;

typedef enum {
    RSP_C64 = 0,        /* complex float32, interleaved re,im */
    RSP_C128 = 1,       /* complex float64, interleaved (MATLAB R2018a mxGetComplexDoubles) */
    RSP_C32F16 = 2      /* complex float16, interleaved (fp16 I/Q, fp32 compute) */
} rsp_dtype;

typedef enum {
    RSP_ROWMAJOR = 0,   /* [P][R]: one pulse (PRT) per row, range contiguous */
    RSP_COLMAJOR = 1    /* MATLAB P x R: [R][P], pulses contiguous */
} rsp_layout;

typedef enum {
    RSP_SEG_FIR = 0,    /* y = scale * filter(taps, 1, x) then circshift(y, -fir_shift)
                           (MTD/fun_lss_pulse_compression.m:38-51) */
    RSP_SEG_MF = 1      /* y[n] = sum_k x[n+k] * conj(s[k]), x zero past in_len and
                           periodic with period nfft (circular when in_len == nfft):
                           MTD/fun_pulse_compression.m:10-39 (linear, nfft >= in_len +
                           coef_len - 1) or DMX_SignalProcessing_main_xzr.m:348-352 */
} rsp_seg_kind;

typedef enum {
    RSP_WIN_KAISER = 0,   /* kaiser(P, window_beta)  (MTD/fun_Process_MTD.m:17-18) */
    RSP_WIN_HAMMING = 1,  /* hamming(P)  (DMX_SignalProcessing_main_xzr.m:211) */
    RSP_WIN_RECT = 2
} rsp_window;

typedef struct {
    int32_t kind;          /* rsp_seg_kind */
    int32_t fir_shift;     /* FIR: out[n] = z[(n + fir_shift) mod out_len] */
    int64_t in_start;      /* input columns [in_start, in_start + in_len) */
    int64_t in_len;
    int64_t out_start;     /* output columns [out_start, out_start + out_len) */
    int64_t out_len;       /* FIR: out_len == in_len; MF: out_len <= nfft */
    int64_t nfft;          /* MF: FFT length, 2^k or 3*2^k, 64 <= nfft <= 16384 */
    double scale;          /* FIR: output scale (1/1.2 for the v2/legacy short pulse);
                              MF: replica scale */
    int64_t coef_len;      /* FIR: taps (<= RSP_MAX_FIR_TAPS); MF: replica length */
    const double* coef_re; /* FIR taps / MF replica real part (copied at rsp_create) */
    const double* coef_im; /* MF replica imaginary part (NULL = 0) */
} rsp_pc_segment;

typedef struct {
    int64_t P;             /* pulses per CPI: 2^k or 3*2^k, 16 <= P <= 1536 */
    int64_t R;             /* input range bins per pulse */
    int64_t R_out;         /* output range bins (PC output = RDM columns) */
    int32_t nseg;          /* pulse-compression segments (<= RSP_MAX_SEG) */
    int32_t window;        /* rsp_window for the slow-time FFT */
    double window_beta;    /* kaiser beta (8 in fun_Process_MTD) */
    int32_t fftshift;      /* 1: fftshift the Doppler axis (fun_Process_MTD.m:31) */
    int32_t zero_v_div;    /* fun_0v_pressing divisor (150 in MTD/fun_0v_pressing.m:22);
                              0 = no suppression */
    rsp_pc_segment seg[RSP_MAX_SEG];
    /* ---- DMX slow-time variant (DMX_SignalProcessing_main_xzr.m:208-229,414-426,462-465);
     *      all zero = the fun_Process_MTD path above ---- */
    int64_t mtd_nfft;      /* Doppler FFT length V (fft(pc.*w, V, 1)); 0 = P.  V > P zero-pads
                              the pulses (DMX mtd_FFT_num = 2048 over prtNum = 1536).  The RDM
                              and the CFAR work on V rows. */
    int32_t beams;         /* 0/1: one beam.  2: the DMX left/right pair -- echo [2][P][R] per
                              CPI (beam 0 = left), RDM = |X_L| + |X_R| (:421-422), optional
                              difference |X_R| - |X_L| (:425-426, rsp_pc_mtd_cfar_diff_dev) */
    int32_t zero_ends;     /* 0: off.  n > 0: zero RDM rows [0, n) and [V-n+1, V) -- the DMX
                              zeroSetFlagMTD with n = MTD_0_num + 1 (:463-465); replaces
                              fun_0v_pressing (zero_v_div) for the RDM */
} rsp_params;

typedef struct {
    int32_t refR, saveR, methodR;   /* range CFAR: reference, guard cells, 0 GO / 1 SO */
    double TR;                      /* range CFAR threshold factor */
    int32_t refV, saveV, methodV;   /* Doppler CFAR */
    double TV;
    int32_t M0;                     /* MTD_0_num: strips rows 1..M0+1 and V-M0+1..V */
    int32_t rFlag;                  /* 1: range CFAR on the Doppler hits; 0: flag = flagV */
    int32_t zero_v_div;             /* fun_0v_pressing before CFAR (20 in
                                       CFAR_WangCai/fun_0v_pressing.m:5); 0 = none */
    int32_t nseg;                   /* column segments; 0 = one segment, all columns */
    int64_t seg_lo[RSP_MAX_SEG];    /* 0-based [seg_lo, seg_hi); columns outside every
                                       segment get flag 0 (main_cfar.m:156-159) */
    int64_t seg_hi[RSP_MAX_SEG];
} rsp_cfar_params;

/* Library version string, e.g. "rsp-mi355x 0.1.0 (gfx950)". */
const char* rsp_version(void);

/* Create a context bound to HIP device `device` for one parameter set.  Builds the
 * matched-filter spectra (fp64 on the host, stored fp32), twiddle tables and window.
 * params == NULL creates a CFAR-only context (rsp_cfar / rsp_cfar_dev). */
int rsp_create(rsp_ctx** out, int device, const rsp_params* params);

/* Context for fun_MTD_produce v2 built from its `params` fields (MTD/fun_MTD_produce.m:
 * 34-69, MTD/main_produce_dataset_win_xzr_v2.m:31-45): P = prtNum, R = echo width,
 * point_prt = {total, p1, p2, p3}, fs [Hz], B [Hz], tao = {tau1, tau2, tau3} [s].
 * Synthesises pulse2 = exp(j*pi*(-B/tau2)*t^2) and pulse3 = exp(j*pi*(B/tau3)*t^2) with
 * t = -tau/2 : 1/fs : tau/2-1/fs, the 35-tap FIR /max /1.2 with its 17-sample group-delay
 * circshift, kaiser(P, 8) + fftshift MTD and fun_0v_pressing /150. */
int rsp_create_v2(rsp_ctx** out, int device, int64_t P, int64_t R, const int64_t point_prt[4],
                  double fs, double B, const double tao[3]);
/* Context for the legacy one-argument MTD_Signal = fun_MTD_produce(echo)
 * (MatlabProcess_xuzerui/fun_MTD_produce.m:3-126; called at main_produce_dataset_win_xzr.m:37-38):
 * P = prtNum, R = echo width, the hard-coded split 82 / 242 / R-324 (:24-38), the 35-tap FIR
 * /max /1.2 with no group-delay shift, the two measured pulses the .m file holds inline
 * (pulse2: n2 samples, pulse3: n3 samples, as separate real / imaginary arrays -- the shim
 * reads them from the repository's data files), kaiser(P, 8) + fftshift MTD, 0-v /150. */
int rsp_create_legacy(rsp_ctx** out, int device, int64_t P, int64_t R, const double* pulse2_re,
                      const double* pulse2_im, int64_t n2, const double* pulse3_re, const double* pulse3_im,
                      int64_t n3);
int rsp_destroy(rsp_ctx* ctx);
const char* rsp_last_error(const rsp_ctx* ctx);

/* CPIs processed per internal chunk (PC scratch = chunk * P * R_out * 8 bytes, sized to
 * stay in the 256 MiB Infinity Cache).  0 restores the default.  Window mode counts output
 * windows: chunk / windows frame pairs per chunk (each chunk also pulse-compresses one
 * look-ahead frame); the default there is at least 32 pairs (fewer look-ahead frames and
 * launches beat Infinity-Cache residency for the window stream). */
int rsp_set_chunk(rsp_ctx* ctx, int64_t cpis_per_chunk);

/* Number of chunk pipelines (1..4; 0 = the default: 2, window mode 1): chunk k runs on the
 * caller's stream or on one of n-1 context-owned streams that fork from and join back into
 * it, so consecutive chunks overlap.  Each pipeline owns one PC scratch slot (n = 1: every
 * launch alone, for per-kernel timing). */
int rsp_set_streams(rsp_ctx* ctx, int32_t n);

/* Device memory a chain context holds (grow-only pools, freed by rsp_destroy), per call shape:
 *   PC scratch        pipelines x chunk x beams x P x R_out x 8 B (c3: 2 x 16 x 128 x 4096 x 8 = 128 MiB)
 *   hit-list slots    the grouped range stage keeps up to 16 chunks' Doppler-hit lists per
 *                     pipeline, each MTD workgroup's region sized to its own cells (no overflow
 *                     possible): pipelines x 16 x chunk x V x R_out x 4 B, capped at 1 GiB
 *                     (c3: exactly 1 GiB; c5, one-CPI chunks: 2 x 16 x 32 MiB = 1 GiB)
 *   host-call staging the host-buffer entry points' device copies of their inputs / outputs
 * i.e. ~1.2 GiB per context at c3, against 288 GB of HBM; rsp_set_chunk scales all three. */

/* ---- host-buffer entry points (MEX / fun_MTD_produce drop-in), synchronous ---------- */
/* rsp_pc_mtd_cfar / rsp_pc_mtd take pageable host buffers (MATLAB's arrays).  A call that fits
 * one chunk (every MATLAB-granularity call) is staged through pinned memory that the kernels
 * read and write directly across PCIe: the host copy threads convert ~1 MiB input pieces while
 * the transpose kernels consume the earlier ones, and deliver ~1 MiB output parts while the later
 * parts cross the link.  A larger batch is pipelined in chunks of CPIs: chunk k's host->device
 * copy, chain and device->host copy overlap chunks k+1 and k-1 (two copy streams beside the
 * context's stream), staged through rings of 8 MiB pinned pieces copied by the thread pool.
 * Outputs are identical to the _dev path's. */
/* CPIs per host chunk (0 = by size: 32 MiB of device-side input, 8 CPIs at 128 x 4096) and
 * host copy threads (0 = default: 8 with >= 16 hardware threads). */
int rsp_set_host_pipeline(rsp_ctx* ctx, int64_t cpis_per_chunk, int32_t copy_threads);

int rsp_pc_mtd(rsp_ctx* ctx, const void* echo, int32_t dtype, int32_t layout,
               int64_t P, int64_t R, int64_t batch, float* rdm_out, int32_t rdm_layout);

int rsp_cfar(rsp_ctx* ctx, const float* rdm, int32_t rdm_layout, int64_t V, int64_t R,
             int64_t batch, const rsp_cfar_params* cfar, uint8_t* flag_out,
             uint8_t* flagV_out /* nullable */);

int rsp_pc_mtd_cfar(rsp_ctx* ctx, const void* echo, int32_t dtype, int32_t layout,
                    int64_t P, int64_t R, int64_t batch, const rsp_cfar_params* cfar,
                    float* rdm_out /* nullable */, int32_t out_layout, uint8_t* flag_out,
                    uint8_t* flagV_out /* nullable */);

/* MATLAB-typed forms for the MEX drop-ins (replacing the .m functions' own double outputs,
 * MTD/fun_MTD_produce.m:12 and CFAR_WangCai/executeCFAR.m:1-2): as rsp_pc_mtd_cfar / rsp_cfar,
 * but the RDM and the 0/1 flags land as double and the CFAR input is double.  The widening
 * (float -> double, byte -> double) and narrowing (double -> float, round to nearest) run on
 * the host copy threads, piece by piece as each pinned piece or part lands, instead of in a
 * serial loop in the shim.  Values are identical to the float / byte forms'.  rsp_pc_mtd_cfar_f64
 * with cfar == NULL is fun_MTD_produce. */
int rsp_pc_mtd_cfar_f64(rsp_ctx* ctx, const void* echo, int32_t dtype, int32_t layout,
                        int64_t P, int64_t R, int64_t batch, const rsp_cfar_params* cfar,
                        double* rdm_out /* nullable */, int32_t out_layout, double* flag_out,
                        double* flagV_out /* nullable */);
int rsp_cfar_f64(rsp_ctx* ctx, const double* rdm, int32_t rdm_layout, int64_t V, int64_t R,
                 int64_t batch, const rsp_cfar_params* cfar, double* flag_out,
                 double* flagV_out /* nullable */);

/* ---- device-pointer entry points, asynchronous on `stream` -------------------------- */
/* d_echo: [batch][P][R] rsp_dtype RSP_C64 or RSP_C32F16.  cfar == NULL: PC + MTD only.
 * d_rdm may be NULL only when cfar != NULL (then an internal buffer is used). */
int rsp_pc_mtd_cfar_dev(rsp_ctx* ctx, const void* d_echo, int32_t dtype, int64_t batch,
                        const rsp_cfar_params* cfar, float* d_rdm, uint8_t* d_flag,
                        uint8_t* d_flagV, void* stream);

int rsp_cfar_dev(rsp_ctx* ctx, const float* d_rdm, int64_t V, int64_t R, int64_t batch,
                 const rsp_cfar_params* cfar, uint8_t* d_flag, uint8_t* d_flagV,
                 void* stream);

/* The chain after pulse compression (fun_Process_MTD + fun_0v_pressing + executeCFAR) on
 * already pulse-compressed rows, e.g. from rsp_pc_dev: d_pc [batch][beams][P][R_out] RSP_C64.
 * Outputs as rsp_pc_mtd_cfar_dev. */
int rsp_mtd_cfar_dev(rsp_ctx* ctx, const void* d_pc, int64_t batch, const rsp_cfar_params* cfar,
                     float* d_rdm, uint8_t* d_flag, uint8_t* d_flagV, void* stream);

/* rsp_pc_mtd_cfar_dev for a two-beam context (rsp_params.beams == 2): d_echo
 * [batch][2][P][R]; d_sum [batch][V][R_out] = |X_L| + |X_R| (the RDM, zeroSetFlagMTD
 * applied); d_diff (nullable) = |X_R| - |X_L|; CFAR runs on the sum
 * (DMX_SignalProcessing_main_xzr.m:414-472). */
int rsp_pc_mtd_cfar_diff_dev(rsp_ctx* ctx, const void* d_echo, int32_t dtype, int64_t batch,
                             const rsp_cfar_params* cfar, float* d_sum, float* d_diff,
                             uint8_t* d_flag, uint8_t* d_flagV, void* stream);

/* Sliding-window stream (MTD/main_produce_dataset_win_xzr_v2.m:94-144; replaces its
 * beam x window loop of fun_MTD_produce calls at :117-136).  d_frames: [beams][frames+1][P][R]
 * consecutive frames of each beam.  For frame pair (n, n+1) and window i < win, the CPI is rows
 * [s_i, s_i + P) of [frame n; frame n+1] with s_i = round(i*P/win) (0-based, :123).  Outputs
 * [beams][frames][win][P][R_out] (MTD_win_all_beams{b}(i+1,:,:) per frame, :131-139); with
 * cfar != NULL each window also runs executeCFAR (flags in the same layout).  Pulse
 * compression is row-wise, so each frame's PC is computed once and shared by its windows
 * (exact).  win <= 16. */
int rsp_window_pc_mtd_cfar_dev(rsp_ctx* ctx, const void* d_frames, int32_t dtype, int64_t beams,
                               int64_t frames, int32_t win, const rsp_cfar_params* cfar,
                               float* d_rdm, uint8_t* d_flag, uint8_t* d_flagV, void* stream);

/* Pulse compression alone (fun_lss_pulse_compression), for tests and staged use:
 * d_pc = [batch][P][R_out] complex float32. */
int rsp_pc_dev(rsp_ctx* ctx, const void* d_echo, int32_t dtype, int64_t batch, void* d_pc,
               void* stream);

/* ---- execution strategy ------------------------------------------------------------------ */
/* Overlap-save split of long matched filters (default on): a segment whose FFT exceeds 4096
 * points, with no output that wraps, runs as 2048..8192-point overlap-save blocks instead of
 * one whole-length transform (the same correlation sums; results differ by fp32 rounding).
 * enable = 0 selects the whole-length transforms.  The threshold is fixed (4096 points).
 * RSP_ERR_UNSUPPORTED on a context without the specialised PC kernels (nothing to select). */
int rsp_set_pc_split(rsp_ctx* ctx, int32_t enable);

/* Range concatenation between pulse compression and the MTD, replacing
 *   Echo_0 = fun_lss_range_concate(prtNum, Echo_0)
 * (MatlabProcess_xuzerui/fun_lss_range_concate.m:4-7, called at main.m:210-211 -- and commented
 * out in the legacy fun_MTD_produce.m:70): after pulse compression, each row becomes the
 * concatenation of its columns [src_start[i], src_start[i] + len[i]), i < nparts, in order; the
 * MTD, the CFAR and every output then have R_out = sum(len) columns (rsp_pc_dev returns the
 * concatenated rows, rsp_mtd_cfar_dev takes them).  The reference's ranges are
 * {0, 89, 481} / {82, 236, 550} (1-based 1:82, 90:325, 482:1031 of the 1031 PC columns ->
 * 868, the width fun_CFARflag's hard-coded 1:82 | 83:318 | 319:868 split assumes,
 * main_cfar.m:143-145).  nparts = 0 restores the PC width.  Parts must lie inside the
 * params' R_out columns; nparts <= RSP_MAX_SEG. */
int rsp_set_range_concat(rsp_ctx* ctx, int32_t nparts, const int64_t* src_start, const int64_t* len);

/* ---- raw-data ingest --------------------------------------------------- */
/* One frame of the radar's PRT record stream -> DBF beams, replacing the per-PRT loop of
 *   [sig_data_DBF_allprts, servo_angle, frameCompleted, is_global_stream_end] =
 *       FrameDataRead_xzr(orgDataFilePath, DBF_coeffs_data_C, Sig_Config, frameRInd)
 * (FrameDataRead_xzr.m:20-204, called at bin_to_mat_xzr.m:62).  The host reads the frame's
 * bytes from the cross-file stream (read_continuous_file_stream.m; rsp/ingest.py mirrors it)
 * and this call parses and beamforms them on the GPU.  Record = head (bytes_head, uint32
 * fields), realtime block, payload padded to 64 B (DDC: int16 I/Q [sample][channel][I,Q]),
 * tail; in rsp_ingest_ddc_dev every PRT has the DDC record size (rsp_ingest_record_bytes).
 * Output (DDC): d_out[b * beam_stride + prt * point_prt + s] = sum_c (I + jQ)[s][c] * dbf[b][c]
 * (sig_data_C * DBF_coeffs_data_C.', :158) as complex64, beam-major so each beam is the
 * [prt][sample] echo the chain reads; beam_stride = 0 means prt_num * point_prt (pass a larger
 * stride to land frames in a [beam][frames+1][P][R] window buffer).
 * d_status: int32[prt_num + 1], per-PRT RSP_PRT_* codes, and [prt_num] = rows decoded: the
 * frame stops at the first PRT the reference would return at (those rows and all later ones
 * are written as zeros, servo 0), so frameCompleted == (status[prt_num] == prt_num && no
 * RSP_PRT_TAIL_TRUNCATED).  rsp_ingest_ddc_dev decodes DDC payloads (data_type 1) only, every
 * record sized by the params; rsp_ingest_frame_dev decodes every data type the reference
 * parses, each record sized by its own head (:104-119), so a frame may mix types:
 *   ADC (0): the int16 (samples x channels) matrix itself (:144-147) -- passes the size check
 *            only with channel_num (of the head) == beam_num; beam b = (x_b, 0);
 *   DBF (any other type): the 24-bit branch (:130-135,162-164) as MATLAB evaluates it -- its
 *            data_temp is uint8, so b0 + b1*2^8 + b2*2^16 saturates to 255 once b1 or b2 is
 *            non-zero (else b0) and the sign fix never fires; beam b = (v_2b, v_2b+1).  The
 *            sizes pass only when the value count (2*ch for ch % 4 == 1, 2*ch + 2 for
 *            ch % 4 == 0) is 2*beam_num; other channel counts are a MATLAB size error there and
 *            RSP_PRT_BAD_SHAPE here.  (The reference marks this branch unfinished.)
 * The two calls share per-context scratch: one frame at a time per context. */
typedef struct {
    int32_t prt_num;         /* Sig_Config.prtNum (332) */
    int32_t point_prt;       /* Sig_Config.point_PRT (3404) */
    int32_t channel_num;     /* Sig_Config.channel_num (16) */
    int32_t beam_num;        /* Sig_Config.beam_num (13) */
    int32_t bytes_head;      /* Sig_Config.bytesFrameHead (64) */
    int32_t bytes_realtime;  /* Sig_Config.bytesFrameRealtime (128) */
    int32_t bytes_tail;      /* Sig_Config.bytesFrameEnd (64) */
} rsp_ingest_params;

enum {
    RSP_PRT_OK = 0,
    RSP_PRT_TRUNCATED = 1,        /* head, realtime block or payload cut by the end of the stream */
    RSP_PRT_TAIL_TRUNCATED = 2,   /* decoded, but the tail is cut: the frame ends incomplete */
    RSP_PRT_BAD_COUNT = 3,        /* pulse_data_num <= 0 (FrameDataRead_xzr.m:90-94) */
    RSP_PRT_BAD_SHAPE = 4,        /* pulse_data_num != point_prt or channels != channel_num */
    RSP_PRT_UNSUPPORTED_TYPE = 5  /* data_type != 1 (DDC) in rsp_ingest_ddc_dev */
};

/* Bytes of one DDC PRT record of this shape. */
int rsp_ingest_record_bytes(const rsp_ingest_params* p, int64_t* bytes);
/* d_stream: nbytes of the frame's records (fewer than prt_num records: the rest are
 * truncated); d_dbf: float32 [beam_num][channel_num][2] (re, im); d_servo nullable. */
int rsp_ingest_ddc_dev(rsp_ctx* ctx, const uint8_t* d_stream, int64_t nbytes, const rsp_ingest_params* p,
                       const float* d_dbf, void* d_out, int64_t beam_stride, uint16_t* d_servo,
                       int32_t* d_status, void* stream);
/* Every data type, records sized by their heads (the same arguments; d_dbf is read by DDC
 * records only). */
int rsp_ingest_frame_dev(rsp_ctx* ctx, const uint8_t* d_stream, int64_t nbytes, const rsp_ingest_params* p,
                         const float* d_dbf, void* d_out, int64_t beam_stride, uint16_t* d_servo,
                         int32_t* d_status, void* stream);

/* ---- post-detection measurement --------------------------------------- */
/* Range / velocity / elevation of every CFAR hit, replacing
 *   [rEstSeries, vEstSeries, eleAngleEstSeries] = motionParaMeasure(echo_MTD_sum, echo_MTD_diff,
 *       cfarResultFlag, extraDots, rScale, deltaR, rInterpTimes, vScale, deltaV, vInterpTimes,
 *       kValues, beamPosNum, beamAngleStep, freInd, eleAngleComp, eleAngleSysErr, MTD_0_num)
 * (MatlabProcess_xuzerui/CFAR_WangCai/motionParaMeasure.m:1-88, called at
 * DMX_SignalProcessing_main_xzr.m:489-494) for a batch of CPIs.  d_sum / d_diff: float32
 * [batch][V][R] (rsp_pc_mtd_cfar_diff_dev's d_sum / d_diff), d_flag: uint8 [batch][V][R]
 * (its d_flag); d_r_scale: float64 [R] (rScale), d_v_scale: float64 [V] (vScale).
 * Hit i of a CPI, in MATLAB's find() order (column-major: range bin, then Doppler row), gets
 * d_est[(cpi*max_hits + i)*3 + {0,1,2}] = {rEst, vEst, eleAngleEst} (float64) and, when
 * d_cells != NULL, d_cells[(cpi*max_hits + i)*2 + {0,1}] = its 0-based (row, column).
 * d_count[cpi*2] = hits in the CPI (only the first max_hits are written), d_count[cpi*2+1] =
 * hits the reference stops at with an index error (a hit too close to an edge for the
 * re-anchoring at :24-32 / :51-59); their estimates are NaN.  With mp->ld > R the three
 * planes are R-column windows of rows ld elements apart. */
typedef struct {
    int32_t extra_dots;      /* extraDots (2), 1..4: 2*extraDots+1 cells per spline */
    int32_t r_interp;        /* rInterpTimes (8), 1..64 */
    int32_t v_interp;        /* vInterpTimes (4), 1..64 */
    int32_t mtd0_num;        /* MTD_0_num: rows 1..M0+1 and V-M0+1..V are clutter-zeroed */
    int32_t beam_pos_num;    /* beamPosNum */
    double delta_r;          /* deltaR [m] */
    double delta_v;          /* deltaV [m/s] */
    double k_value;          /* kValues(freInd+1, beamPosNum+1) (angle_KvalueGen.m) */
    double beam_angle_step;  /* beamAngleStep [deg] (5) */
    double ele_comp;         /* eleAngleComp */
    double ele_sys_err;      /* eleAngleSysErr */
    int64_t ld;              /* row pitch of the planes in elements (0 = R): a column window of a
                                wider plane, e.g. DMX's short part (columns 0..61) or long part
                                (62..573, pass the planes + 62) measured separately as the
                                reference does (DMX_SignalProcessing_main_xzr.m:489-494) */
    int64_t cpi_stride;      /* elements between CPIs (0 = V * ld) */
} rsp_measure_params;

int rsp_motion_measure_dev(rsp_ctx* ctx, const float* d_sum, const float* d_diff, const uint8_t* d_flag,
                           int64_t V, int64_t R, int64_t batch, const rsp_measure_params* mp,
                           const double* d_r_scale, const double* d_v_scale, int64_t max_hits,
                           double* d_est, int32_t* d_cells /* nullable */, int32_t* d_count, void* stream);

/* ---- echo pre-filters ---------------------------------------------------- */
/* iSTC and MTI on a device-resident echo batch, complex64 [batch][P][R] (row = pulse, the
 * chain's ROWMAJOR layout), before pulse compression:
 *   d_gain != NULL: out(m, n) *= d_gain[n], the linear gain 10^(stc(n)/20) of
 *       [stc, eoch_iSTC] = fun_iSTC(echo)            (MTD/fun_iSTC.m:12-15; the caller reads
 *       the stc curve and zero-pads it to R as :8-9 do -- rsp/prefilter.py istc_gain);
 *   mti_lag > 0: out(m, :) = x(m+lag, :) - x(m, :) for m < P-lag, 0 for the last lag rows,
 *       MTI_Out = fun_Process_MTI(ProSiganl)          (MTD/fun_Process_MTI.m:9,20-22; lag 30).
 * Both: the MTI difference first, then the gain (the two commute up to fp32 rounding).
 * R must be even and d_in / d_out 16-byte aligned; d_out == d_in is allowed only without MTI. */
int rsp_prefilter_dev(rsp_ctx* ctx, const void* d_in, void* d_out, int64_t P, int64_t R, int64_t batch,
                      const float* d_gain /* nullable, [R] */, int32_t mti_lag, void* stream);

/* The same pre-filters fused into the context's chain (every rsp_pc_mtd*, rsp_run*, window
 * entry point after this call), with no pass of their own over the echo:
 *   gain != NULL (host, [R] linear gains as above): applied to each echo sample as pulse
 *       compression loads it (needs the per-segment PC kernels -- the v2, dmx and legacy
 *       presets; RSP_ERR_UNSUPPORTED otherwise);
 *   mti_lag > 0: applied to the pulse-compressed rows as the MTD loads them -- pulse
 *       compression is linear per row, so PC(x(m+lag) - x(m)) = PC(x(m+lag)) - PC(x(m)) --
 *       over the pulses of each CPI (each window in window mode), zero for its last lag rows.
 * gain == NULL and mti_lag == 0 switch the fused pre-filters off.
 * rsp_pc_dev (pulse compression alone) applies the gain but not MTI, which lives in the MTD
 * stage: its rows are PC(gain .* x). */
int rsp_set_prefilter(rsp_ctx* ctx, const float* gain /* nullable, host [R] */, int32_t mti_lag);

/* ---- diagnostics ---------------------------------------------------------------------- */
/* Per-kernel device time accumulated from HIP events recorded on the launch stream around
 * kernel launches while profiling is enabled: enable = 1 brackets every launch, enable = N > 1
 * every N-th launch (sampling: each event pair costs the stream a few microseconds),
 * 0 stops.  Any call resets the counters.
 * Kernel ids: RSP_K_PC, RSP_K_MTD, RSP_K_CFAR_R, RSP_K_CFAR_V. */
#define RSP_NKERNELS 4
enum { RSP_K_PC = 0, RSP_K_MTD = 1, RSP_K_CFAR_R = 2, RSP_K_CFAR_V = 3 };
int rsp_profile(rsp_ctx* ctx, int32_t enable);
/* Waits for the recorded events; ms[k] = summed device time, launches[k] = launch count, for
 * k < n (n <= RSP_NKERNELS entries are written; pass the length of both arrays). */
int rsp_profile_read_n(rsp_ctx* ctx, double* ms, int64_t* launches, int32_t n);
/* ABI-3 form: writes exactly 4 entries (RSP_K_PC .. RSP_K_CFAR_V), whatever RSP_NKERNELS is. */
int rsp_profile_read(rsp_ctx* ctx, double* ms, int64_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* RSP_H */
