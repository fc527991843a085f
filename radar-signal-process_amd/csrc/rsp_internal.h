// rsp_internal.h -- argument blocks shared by the C-ABI host code (rsp_capi.cpp) and the
// HIP kernels (rsp_kernels.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

#include "../../include/rsp.h"

namespace rsp {

constexpr int kBlock = 256;  // threads per workgroup for every kernel (4 waves of 64)

// One-time launch setup of a kernel (hipFuncSetAttribute, occupancy -> resident grid), per
// device: both apply to the calling thread's current device, and contexts on different host
// threads and devices launch concurrently (rsp.h threading model), so the setup runs once per
// (kernel, device) under std::call_once and its result is cached per device.
constexpr int kMaxDevices = 64;
struct LaunchOnce {
    std::once_flag once[kMaxDevices];
    hipError_t err[kMaxDevices] = {};
    int value[kMaxDevices] = {};
};
// init(dev, &value) -> hipError_t; *value receives the cached value (e.g. resident workgroups)
template <typename F>
inline hipError_t launch_once(LaunchOnce& L, int* value, F&& init) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= kMaxDevices) return hipErrorInvalidDevice;
    std::call_once(L.once[dev], [&] { L.err[dev] = init(dev, &L.value[dev]); });
    if (value) *value = L.value[dev];
    return L.err[dev];
}

// One pulse-compression segment as the kernel sees it (see rsp_pc_segment).
struct SegDev {
    int kind;        // RSP_SEG_FIR / RSP_SEG_MF
    int fir_shift;
    int in_start, in_len;
    int out_start, out_len;
    int nfft;
    int ntaps;
    float scale;
    const float2* H;   // MF: conj(FFT_nfft(scale*replica)) / nfft
    const float2* tw;  // MF: W_nfft^e table, e < nfft
    const float* taps_dev;  // FIR taps in device memory (no dynamic kernarg indexing)
    int ntaps4;             // ntaps rounded up to a multiple of 4
    const float2* taps2_dev;  // (scale*b_k, scale*b_k), zero-padded to ntaps4: one packed fma per tap
    float taps[RSP_MAX_FIR_TAPS];
};

struct PcArgs {
    int P, R, R_out;
    int nseg;
    int nzero;                          // output column ranges no segment writes
    int zero_lo[RSP_MAX_SEG + 1];
    int zero_hi[RSP_MAX_SEG + 1];
    SegDev seg[RSP_MAX_SEG];
};

// One matched-filter segment for every row, specialised on its FFT length; the first
// launch of a chunk also runs the FIR segment and zero-fills uncovered columns.
struct PcMfArgs {
    int R, R_out;
    int rows;
    int do_fir;
    SegDev fir;
    SegDev mf;
    // overlap-save split of a long matched filter (nsub > 1): sub-block j of a row correlates
    // input [in_start + j*sub_step, + mf.nfft) with the replica (mf.H, mf.nfft points) and keeps
    // outputs [j*sub_step, (j+1)*sub_step) -- sub_step = mf.nfft - replica length + 1, so no
    // output wraps.  nsub <= 1: the whole segment in one mf.nfft-point transform.
    int nsub, sub_step;
    const float* gain;   // fused iSTC (rsp_set_prefilter): echo column n scaled by gain[n], or null
    int nzero;
    int zero_lo[RSP_MAX_SEG + 1];
    int zero_hi[RSP_MAX_SEG + 1];
};

// Doppler-dimension CFAR on one column tile (Function_CFAR1D_sub on used.').
struct CfarVArgs {
    int enabled;
    int lo, hi;          // used rows [lo, hi) = rows M0+2 .. V-M0 (1-based)
    int ref, save, method;
    float T;
    float Tr;            // T / ref (threshold = max|min(window sums) * Tr)
    int cz_lo, cz_hi;    // rows zeroed before CFAR (main_cfar.m:90-91), empty if lo >= hi
    int nseg;            // column segments (fun_CFARflag); columns outside get flag 0
    int seg_lo[RSP_MAX_SEG], seg_hi[RSP_MAX_SEG];
};

// Range-dimension CFAR at the Doppler hits (executeCFAR.m:35-89).
struct CfarRArgs {
    int V, R;
    int lo, hi;          // used rows
    int rflag;
    int ref, save, method;
    float T;
    float Tr;            // T / ref
    int cz_lo, cz_hi;    // rows zeroed before CFAR
    int nseg;
    int seg_lo[RSP_MAX_SEG], seg_hi[RSP_MAX_SEG];
};

constexpr int RSP_MAX_WIN = 16;

struct MtdArgs {
    int P, R_out;
    // Sliding-window mode (main_produce_dataset_win_xzr_v2.m:117-131): launch CPI j is window
    // j % nwin of frame j / nwin; its P pulses are PC rows [n*P + win_start[j % nwin], +P) of
    // a frame-contiguous PC buffer.  nwin == 0: CPI j reads rows [j*P, (j+1)*P).
    int nwin;
    int win_start[RSP_MAX_WIN];
    int pin;             // pulses per CPI and beam (<= P; the FFT zero-pads rows pin..P-1)
    int mti_lag;         // fused MTI (rsp_set_prefilter): pulse p reads row p+lag minus row p, 0 past pin-lag
    int beams;           // 2: DMX pair -- RDM = |X_0| + |X_1|, diff (if non-null) = |X_1| - |X_0|
    float* diff;
    // Bluestein plan for P without a radix plan (v2 native P = 332): bnf > 0 is the power-of-
    // two convolution length, bwc[n] = w[n] exp(-j pi n^2/P) (0 for n >= P), bspec = FFT of the
    // conjugate chirp / bnf; tw is then the bnf-point twiddle table.
    int bnf;
    const float2* bwc;
    const float2* bspec;
    int shift;           // fftshift offset floor(P/2), or 0
    int z_lo, z_hi;      // fun_0v_pressing rows zeroed in the RDM
    const float* win;    // slow-time window, P entries
    const float2* tw;    // W_P^e table
    CfarVArgs cv;
    // Fused range-CFAR front end (cv.enabled): the MTD kernel writes the final flag plane's
    // background -- flagV itself when rflag == 0, zeros otherwise -- and appends every
    // in-band Doppler hit (linear cell index within the launch) to `hits`; cfar_hits_kernel
    // then sets the re-localised range detections.  flagV is written only when requested.
    uint8_t* flag;
    int rflag;
    int flag_zero;         // rflag: the MTD kernel writes the flag plane's zeros (else the host memsets it)
    uint32_t* hits;        // workgroup b owns hits[b*W*P, (b+1)*W*P) (its own cells: no overflow)
    uint32_t* hit_count;   // hit_count[b] = entries of workgroup b (b = blockIdx.y*gridDim.x + blockIdx.x)
    uint32_t cell_off;     // added to every hit index (grouped range stages: the chunk's offset in its group)
    // The previous chunk's range stage, run by extra workgroups of this launch (same stream,
    // so that chunk's RDM and hit lists are complete): prev_nregions == 0 means none.
    const float* prev_rdm;
    uint8_t* prev_flag;
    const uint32_t* prev_hits;
    const uint32_t* prev_count;
    int prev_nregions, prev_region;
    CfarRArgs prev_cr;
};


// Raw-data ingest (rsp_ingest.hip): one frame of uniform DDC PRT records.
// motionParaMeasure.m's scalar arguments (rsp_measure_params, rsp_measure.hip).
struct MeasureArgs {
    int extra_dots, r_interp, v_interp, mtd0_num, beam_pos_num;
    double delta_r, delta_v, k_value, beam_angle_step, ele_comp, ele_sys_err;
    int64_t ld, cs;   // row pitch and CPI stride of the planes, in elements
};
// Workgroups per CPI for the hit lists (1: hits_kernel; > 1: the banded path, which needs
// batch * nb * R int32 of scratch in band_cnt).
int measure_bands(int V, int batch);
hipError_t launch_measure(const float* sum, const float* diff, const uint8_t* flag, int V, int R, int batch,
                          const MeasureArgs& a, const double* r_scale, const double* v_scale, int64_t max_hits,
                          double* est, int32_t* cells, int32_t* count, int32_t* band_cnt, int nb, hipStream_t st);

// Echo pre-filters (rsp_prefilter.hip): iSTC gain per range bin and/or MTI row difference.
hipError_t launch_prefilter(const float2* in, float2* out, const float* gain, int P, int R, int64_t batch, int lag,
                            hipStream_t st);

struct IngestArgs {
    int prt_num, point_prt, channel_num, beam_num;
    int bytes_head, bytes_realtime, bytes_tail;
    int64_t rec_bytes;       // head + realtime + payload (padded to 64 B) + tail of a DDC record
    int64_t beam_stride;     // output elements between consecutive beams' [prt][sample] planes
    int ddc_only;            // rsp_ingest_ddc_dev: records sized by the params, other types refused
    int64_t* offs;           // [prt_num] record offsets in the stream (check -> decode kernel)
    int32_t* types;          // [prt_num] data types of the decoded records
    int dbf_lds;             // (launch_ingest) generic-shape decode: the DBF matrix staged in LDS
};
hipError_t launch_ingest(const uint8_t* stream, int64_t nbytes, const IngestArgs& a, const float2* dbf,
                         float2* out, uint16_t* servo, int32_t* status, hipStream_t s);

// Payload bytes of one record by data type (FrameDataRead_xzr.m:104-119): ADC (0) int16 per
// channel, DDC (1) int16 I/Q per channel, anything else the 24-bit DBF layout (3-byte I/Q per
// channel plus 8 - mod(6*ch, 8) pad bytes per sample), the whole padded to 64 B.
constexpr int64_t ingest_payload_bytes(uint32_t type, int64_t pdn, int64_t ch) {
    const int64_t sig = type == 0 ? pdn * ch * 2
                      : type == 1 ? pdn * ch * 4
                                  : pdn * ch * 6 + pdn * (8 - (6 * ch) % 8);
    return sig % 64 ? sig + 64 - sig % 64 : sig;
}
// 24-bit DBF branch (FrameDataRead_xzr.m:130-135,162-164): bytes per sample row, and the number
// of values the three column ranges 1:3:end-3, 2:3:end-2, 3:3:end give (-1 when their lengths
// differ or the count is odd: the reference's own sum or I/Q pairing raises a size error).
constexpr int dbf24_row_bytes(int ch) { return 6 * ch + (8 - (6 * ch) % 8); }
constexpr int dbf24_values(int ch) {
    const int L = dbf24_row_bytes(ch);
    const int n1 = L - 3 >= 1 ? (L - 4) / 3 + 1 : 0, n2 = L - 2 >= 2 ? (L - 4) / 3 + 1 : 0, n3 = L / 3;
    return (n1 == n2 && n2 == n3 && n1 % 2 == 0) ? n1 : -1;
}

bool mtd_size_supported(int P, int beams = 1);
bool pc_nfft_supported(int n);
size_t pc_lds_bytes(int max_nfft);

hipError_t launch_pc(const void* echo, int dtype, float2* out, int64_t rows, const PcArgs& a,
                     size_t lds_bytes, hipStream_t s);
// float2 slots the FIR stages in the row's LDS slot: ntaps4-1 leading zeros, the segment,
// and the 4-output block's read-ahead
inline int fir_stage_len(const SegDev& g) { return g.ntaps4 - 1 + g.out_len + 4; }
bool pc_mf_supported(int nfft, int fir_stage_len);
bool pc_pair_supported(int nfft1, int nfft2);
// a2 == nullptr: one segment; otherwise both segments (a1.mf.nfft, a2->mf.nfft) in one launch
hipError_t launch_pc_mf(const void* echo, int dtype, float2* out, const PcMfArgs& a1, const PcMfArgs* a2,
                        hipStream_t s);
hipError_t launch_mtd(const float2* pc, float* rdm, uint8_t* flagV, int ncpi, const MtdArgs& a,
                      hipStream_t s);
// Doppler CFAR straight from an RDM ([ncpi][V][R] fp32) for rsp_cfar.
hipError_t launch_cfar_v(const float* rdm, uint8_t* flagV, int ncpi, int V, int R,
                         const CfarVArgs& a, hipStream_t s);
// Range CFAR + re-localisation at the Doppler hits listed by the MTD kernel (scatter form of
// executeCFAR.m:45-84).  `zero_slot` (if non-null) is reset for a later launch.
hipError_t launch_cfar_hits(const float* rdm, uint8_t* flag, const uint32_t* hits, const uint32_t* counts,
                            int nregions, int region, const CfarRArgs& a, hipStream_t s);
// MTD workgroups per launch and cells per workgroup (hit-list regions)
void mtd_regions(int P, int R_out, int ncpi, int* nregions, int* region, int beams = 1);
// Bluestein convolution length for a P without a radix plan (0: unsupported)
int mtd_bluestein_nf(int P);
hipError_t launch_cfar_r(const float* rdm, const uint8_t* flagV, uint8_t* flag, int ncpi,
                         const CfarRArgs& a, hipStream_t s);
// Whether launch_cfar_r has a kernel for the row length / window (the generic kernel stages a
// row in LDS: 10 bytes per cell)
bool cfar_r_supported(const CfarRArgs& a);
// dtype/layout conversion of a host-API input into [batch][P][R] complex float32.
hipError_t launch_ingest(const void* in, int dtype, int layout, float2* out, int64_t batch,
                         int P, int R, hipStream_t s);
// [batch][A][B] -> [batch][B][A] for 4-byte and 1-byte elements.
hipError_t launch_transpose_f32(const float* in, float* out, int64_t batch, int A, int B,
                                hipStream_t s);
hipError_t launch_transpose_u8(const uint8_t* in, uint8_t* out, int64_t batch, int A, int B,
                               hipStream_t s);
// One plane's sub-block transpose: element (a, b), a < A, b < B, of in[a*in_pitch + b] to
// out[b*out_pitch + a] (elements: RSP_SUB_*; C32F16 widens to complex float).  The host path's
// pieces: either pointer may be pinned host memory.
enum { RSP_SUB_F32 = 0, RSP_SUB_U8 = 1, RSP_SUB_C64 = 2, RSP_SUB_C32F16 = 3 };
hipError_t launch_transpose_sub(int elem, const void* in, void* out, int A, int B, size_t in_pitch, size_t out_pitch,
                                hipStream_t s);
// nwords 4-byte words in -> out (either may be pinned host memory)
hipError_t launch_copy_words(const void* in, void* out, size_t nwords, hipStream_t s);

}  // namespace rsp
