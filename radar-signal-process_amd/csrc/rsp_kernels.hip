// rsp_kernels.hip -- the hot path of the range-Doppler chain as gfx950 kernels.
//
//   pc_kernel      one workgroup per pulse (PRT) row: FIR segment(s) + frequency-domain
//                  matched filter segment(s), FFT -> x conj(replica spectrum) -> FFT, all in
//                  LDS.  Restates MTD/fun_lss_pulse_compression.m:17-80 with
//                  fun_pulse_compression.m:10-39 (linear correlation via a power-of-two
//                  FFT, SURVEY.md §8a-3 equivalence) and the DMX circular matched filter
//                  (CFAR_WangCai/DMX_SignalProcessing_main_xzr.m:348-352).
//   mtd_kernel     one workgroup per tile of W range bins x all P pulses: slow-time window,
//                  P-point FFT per range bin, fftshift, |.|, fun_0v_pressing, then the
//                  Doppler-dimension CA-CFAR on the same columns while they sit in LDS
//                  (MTD/fun_Process_MTD.m:13-40, MTD/fun_0v_pressing.m:13-24,
//                   CFAR_WangCai/executeCFAR.m:23-31 with Function_CFAR1D_sub.m:17-69).
//   cfar_r_kernel  one workgroup per RDM row: range-dimension CFAR at the Doppler hits and
//                  the first-argmax re-localisation (executeCFAR.m:35-89,
//                  Function_CFAR1D_sub_fixCells.m:23-87), written as a gather so the output
//                  is deterministic and needs no zero-fill pass.
//   cfar_v_kernel  the Doppler CFAR straight from an RDM (standalone rsp_cfar).
//   ingest / transpose kernels for the host-buffer (MATLAB column-major) entry points.
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <type_traits>

#include "rsp_fft.h"
#include "rsp_buf.h"
#include "rsp_diag.h"
#include "rsp_internal.h"


namespace rsp {


__device__ __forceinline__ float2 ld_c(const float2* p) { return *p; }
__device__ __forceinline__ float2 ld_c(const __half2* p) { return __half22float2(*p); }
__device__ __forceinline__ float2 ld_c(const double2* p) {
    double2 d = *p;
    return make_float2((float)d.x, (float)d.y);
}

// ================================================================== pulse compression
template <int N, typename TIn>
__device__ __forceinline__ void mf_segment(const TIn* __restrict__ x, float2* __restrict__ y,
                                           const SegDev& g, float2* lds, int t) {
    for (int i = t; i < N; i += kBlock) {
        float2 v = make_float2(0.f, 0.f);
        if (i < g.in_len) v = ld_c(x + g.in_start + i);
        lds[pidx(i)] = v;
    }
    __syncthreads();
    fft_lds<N, kBlock>(lds, t, g.tw);
    // Y = conj(X .* H): the inverse FFT as conj(FFT(conj(.))), 1/N folded into H
    for (int i = t; i < N; i += kBlock) lds[pidx(i)] = cconj(cmul(lds[pidx(i)], g.H[i]));
    __syncthreads();
    fft_lds<N, kBlock>(lds, t, g.tw);
    for (int i = t; i < g.out_len; i += kBlock) y[g.out_start + i] = cconj(lds[pidx(i)]);
    __syncthreads();  // lds is reused by the next segment
}

template <typename TIn>
__device__ __forceinline__ void fir_segment(const TIn* __restrict__ x, float2* __restrict__ y,
                                            const SegDev& g, int t) {
    // z[m] = scale * sum_k taps[k] x[m-k] (causal, zero state); out[n] = z[(n+shift) mod len]
    const int len = g.out_len;
    for (int n = t; n < len; n += kBlock) {
        int m = n + g.fir_shift;
        m %= len;
        float ar = 0.f, ai = 0.f;
#pragma unroll 8
        for (int k = 0; k < RSP_MAX_FIR_TAPS; ++k) {
            if (k < g.ntaps && k <= m) {
                const float2 v = ld_c(x + g.in_start + m - k);
                ar = fmaf(g.taps[k], v.x, ar);
                ai = fmaf(g.taps[k], v.y, ai);
            }
        }
        y[g.out_start + n] = make_float2(ar * g.scale, ai * g.scale);
    }
}

template <typename TIn>
__global__ __launch_bounds__(kBlock) void pc_kernel(const TIn* __restrict__ echo,
                                                    float2* __restrict__ out, PcArgs a) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int t = threadIdx.x;
    const size_t row = blockIdx.x;
    const TIn* x = echo + row * (size_t)a.R;
    float2* y = out + row * (size_t)a.R_out;
    for (int z = 0; z < a.nzero; ++z)
        for (int c = a.zero_lo[z] + t; c < a.zero_hi[z]; c += kBlock) y[c] = make_float2(0.f, 0.f);
#pragma unroll
    for (int s = 0; s < RSP_MAX_SEG; ++s) {
        if (s >= a.nseg) break;
        const SegDev& g = a.seg[s];
        if (g.kind == RSP_SEG_FIR) {
            fir_segment(x, y, g, t);
        } else {
            switch (g.nfft) {
                case 64: mf_segment<64>(x, y, g, lds, t); break;
                case 128: mf_segment<128>(x, y, g, lds, t); break;
                case 256: mf_segment<256>(x, y, g, lds, t); break;
                case 512: mf_segment<512>(x, y, g, lds, t); break;
                case 1024: mf_segment<1024>(x, y, g, lds, t); break;
                case 2048: mf_segment<2048>(x, y, g, lds, t); break;
                case 4096: mf_segment<4096>(x, y, g, lds, t); break;
                case 8192: mf_segment<8192>(x, y, g, lds, t); break;
                case 16384: mf_segment<16384>(x, y, g, lds, t); break;
                default: break;  // rejected on the host
            }
        }
    }
}

bool pc_nfft_supported(int n) {
    switch (n) {
        case 64: case 128: case 256: case 512: case 1024: case 2048: case 4096: case 8192:
        case 16384:
            return true;
        default:
            return false;
    }
}

size_t pc_lds_bytes(int max_nfft) { return (size_t)padded_len(max_nfft < 64 ? 64 : max_nfft) * sizeof(float2); }

hipError_t launch_pc(const void* echo, int dtype, float2* out, int64_t rows, const PcArgs& a,
                     size_t lds_bytes, hipStream_t s) {
    if (rows <= 0) return hipSuccess;
    static LaunchOnce once;
    hipError_t e = launch_once(once, nullptr, [](int, int*) {
        hipError_t r = hipFuncSetAttribute((const void*)pc_kernel<float2>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (r == hipSuccess)
            r = hipFuncSetAttribute((const void*)pc_kernel<__half2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    160 * 1024);
        return r;
    });
    if (e != hipSuccess) return e;
    dim3 grid((unsigned)rows), block(kBlock);
    if (dtype == RSP_C64) {
        hipLaunchKernelGGL(pc_kernel<float2>, grid, block, lds_bytes, s, (const float2*)echo, out, a);
    } else if (dtype == RSP_C32F16) {
        hipLaunchKernelGGL(pc_kernel<__half2>, grid, block, lds_bytes, s, (const __half2*)echo, out, a);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}


// ================================================================== pulse compression v2
// One launch per matched-filter segment, specialised on its FFT length N: G threads per
// PRT row (E = N/G elements each, register-resident Stockham passes), RPB rows per
// 256..512-thread workgroup.  Row loads and stores are lane-contiguous (the strided
// element pattern of fft_reg), the spectrum multiply sits between the forward and the
// inverse FFT in registers, and the only LDS traffic is the inter-pass exchange.
template <int N>
struct PcCfg {
    // 16 elements per thread at every length: a 16384-point row is 1024 threads (4 waves per
    // SIMD, 124 VGPRs with the lean twiddles) -- 32 elements at 512 threads took 164..174 VGPRs
    // and left 2 waves per SIMD
    static constexpr int G = N / 16;                       // threads per row
    static constexpr int E = N / G;                             // elements per thread
    static constexpr int RPB = G >= 256 ? 1 : 256 / G;          // rows per workgroup
    static constexpr int T = G * RPB;
    static constexpr int SLOT = padded_len(N);
    static constexpr size_t lds = (size_t)RPB * SLOT * sizeof(float2);
};

// FIR segment of one row (fun_lss_pulse_compression.m:38-51): z = filter(b, 1, x_A) * scale
// (causal, zero initial state), out[n] = z[(n + shift) mod len].  The segment is staged in
// the row's LDS slot behind ntaps4-1 zeros, so z[m] = sum_k b_k s[kp + m - k] needs no
// bounds test.  A thread produces 4 consecutive z and walks the taps 4 at a time: 7 LDS
// reads and 16 packed fmas per step (taps pre-scaled and duplicated as (b, b), so a wave-
// uniform tap multiplies both I and Q in one v_pk_fma_f32).
__device__ __forceinline__ float2 pk_fma(float2 a, float2 b, float2 c) {
    return make_float2(fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y));
}

// The FIR segment's staging loads of a wave-uniform row (G % 64 == 0): the first B*G staged
// samples (zeros before the segment and past in_len come from the buffer range check), issued
// with the row's matched-filter loads so the two share one memory round trip.
constexpr int kFirB = 8;
template <typename TIn, int G>
__device__ __forceinline__ void fir_stage_issue(float2 (&v)[kFirB], const TIn* __restrict__ x, const SegDev& g,
                                                bool valid, int t, int i0) {
    constexpr uint32_t ES = sizeof(TIn);
    const int kp = g.ntaps4 - 1;
    const auto xr = buf_rsrc(x + g.in_start, valid ? (uint32_t)g.in_len * ES : 0u);
#pragma unroll
    for (int q = 0; q < kFirB; ++q) {
        const int j = i0 + q * G - kp;
        v[q] = buf_ld_c((const TIn*)nullptr, xr, j >= 0 ? (uint32_t)j * ES : kOob, 0u);
    }
}

template <typename TIn, int G, int SA = 0, bool WS = false>
__device__ __forceinline__ void fir_row(const TIn* __restrict__ x, float2* __restrict__ y,
                                        const SegDev& g, float* stage, bool valid, int t,
                                        const float* __restrict__ gain, bool st_ok = true,
                                        const float2* pre = nullptr) {
    float2* s2 = reinterpret_cast<float2*>(stage);
    const int kp = g.ntaps4 - 1;
    const int len = g.out_len;
    const int nst = kp + len + 4;
    if constexpr (G % 64 == 0) {
        // The row is wave-uniform: stage through a range-checked buffer resource, 8 loads per
        // thread issued together, so the staging costs one memory round trip instead of one
        // per element step; `pre` holds the first block's loads when the caller issued them.
        const auto gr = buf_rsrc(gain ? gain + g.in_start : nullptr, gain ? (uint32_t)g.in_len * 4u : 0u);
        constexpr int B = kFirB;
        for (int i0 = t; i0 < nst; i0 += B * G) {
            float2 v[B];
            if (pre && i0 == t) {
#pragma unroll
                for (int q = 0; q < B; ++q) v[q] = pre[q];
            } else {
                fir_stage_issue<TIn, G>(v, x, g, valid, t, i0);
            }
            if (gain) {   // fused iSTC (wave-uniform)
#pragma unroll
                for (int q = 0; q < B; ++q) {
                    const int j = i0 + q * G - kp;
                    v[q] = cscale(v[q], buf_ld_f(gr, j >= 0 ? (uint32_t)j * 4u : kOob, 0u));
                }
            }
#pragma unroll
            for (int q = 0; q < B; ++q)
                if (i0 + q * G < nst) s2[i0 + q * G] = v[q];
        }
    } else {
        for (int i = t; i < nst; i += G) {
            const int j = i - kp;
            float2 v = (valid && j >= 0 && j < g.in_len) ? ld_c(x + g.in_start + j) : make_float2(0.f, 0.f);
            if (gain && j >= 0 && j < g.in_len) v = cscale(v, gain[g.in_start + j]);
            s2[i] = v;
        }
    }
    xsync<WS>();
    RSP_STAMP(0, 10, false);
    const float2* __restrict__ taps = g.taps2_dev;
    for (int m0 = 4 * t; m0 < len; m0 += 4 * G) {
        float2 acc[4] = {};
        const float2* p = s2 + kp + m0;     // p[i] = x[m0 + i]
        float2 w[7];                         // w[q] = x[m0 + q - 3 - k]
        // w[4..6] of tap group k+4 are w[0..2] of group k: 4 LDS reads per group instead of 7
        w[4] = p[1];
        w[5] = p[2];
        w[6] = p[3];
        auto group = [&](int k) {
#pragma unroll
            for (int q = 0; q < 4; ++q) w[q] = p[q - 3 - k];
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                const float2 b = taps[k + kk];
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[i] = pk_fma(w[i - kk + 3], b, acc[i]);
            }
            w[6] = w[2];
            w[5] = w[1];
            w[4] = w[0];
        };
        for (int k = 0; k < g.ntaps4; k += 4) group(k);
        RSP_STAMP(0, 11, false);
        if (valid && st_ok) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int m = m0 + i;
                if (m < len) {
                    int n = m - g.fir_shift;
                    if (n < 0) n += len;
                    st_c<SA>(y + g.out_start + n, acc[i]);
                }
            }
        }
    }
    RSP_STAMP(0, 12, false);
    xsync<WS>();
}

// (The long rows' input by LDS-DMA into the exchange slot, round 4's `-DRSP_PC_DMA` A/B, measured
// +0..1 % at c3 and -1.4 % at c5 and is not kept: DESIGN.md §7b; the source is in the history,
// commit e3a7a73.)
typedef __attribute__((address_space(3))) void lds_void;   // an LDS-DMA destination (the MTD tiles)

// One row's matched-filter segment (and optionally its FIR segment) by G threads.
// G >= 64: a row spans whole waves, so the row index is wave-uniform (readfirstlane makes
// that visible to the compiler) and the row's input/output spans are buffer resources in
// SGPRs -- the zero padding beyond in_len, the out_len cut and invalid rows (num_records 0)
// are the hardware range check, with no per-element branch.  G < 64 (N <= 512): rows share
// a wave, so the accesses stay per-lane predicated.
template <typename TIn, int N, int G, int SA = 0, bool WS = false, int EARLY = -1>
__device__ __forceinline__ void pc_row(const TIn* __restrict__ echo, float2* __restrict__ out,
                                       const PcMfArgs& a, int row, int t, float2* buf, int sub = 0) {
    constexpr int E = N / G;
    constexpr bool kUniform = G % 64 == 0;
    // Every global load of the row -- MF input and the whole spectrum slice -- is issued up
    // front, so one memory round trip overlaps the FIR (short rows) and the spectrum arrives
    // during the forward FFT instead of after it (N <= 4096: the 32 extra live VGPRs fit the
    // paired kernel's allocation, which its short-row path already sets; PC 41 -> 39.8 us per
    // 16 CPIs at c3, 39.7 -> 37.8 us per CPI at c5).  8192/16384-point rows keep the spectrum
    // loads after the forward FFT.
    // (EARLY 0 / 1 overrides: the dataflow kernel's long rows load the spectrum late -- its item
    // loop leaves no room for 32 early spectrum registers)
    constexpr bool kEarly = EARLY >= 0 ? EARLY != 0 : (G <= 64 || N <= 4096);
    if constexpr (kUniform) {   // (a VGPR-held offset in a buffer resource means a waterfall loop per access)
        row = __builtin_amdgcn_readfirstlane(row);
        sub = __builtin_amdgcn_readfirstlane(sub);
    }
    const bool valid = row < a.rows;
    const TIn* x = echo + (size_t)diag_pc_src_row(row) * a.R;
    const bool st_ok = valid && !kDiagPcNoStore;
    float2* y = out + (size_t)row * a.R_out;
    int in_start = a.mf.in_start, in_len = a.mf.in_len;
    int out_start = a.mf.out_start, out_len = a.mf.out_len;
    if (a.nsub > 1) {   // overlap-save sub-block (wave-uniform): shifted input and output windows
        const int off = sub * a.sub_step;
        in_start += off;
        out_start += off;
        in_len = max(0, min(in_len - off, N));
        out_len = max(0, min(out_len - off, a.sub_step));
        if constexpr (kUniform) {
            in_len = __builtin_amdgcn_readfirstlane(in_len);
            out_len = __builtin_amdgcn_readfirstlane(out_len);
            in_start = __builtin_amdgcn_readfirstlane(in_start);
            out_start = __builtin_amdgcn_readfirstlane(out_start);
        }
    }
    const float2* __restrict__ tw = a.mf.tw;
    constexpr uint32_t ES = sizeof(TIn);
    const auto hr = buf_rsrc(a.mf.H, (uint32_t)N * 8u);
    float2 u[E];
    const int e0 = t;   // the thread's element offset in each block of G
    constexpr int NW = tw_regs<N, E>() > 0 ? tw_regs<N, E>() : 1;
    float2 w[NW];
    tw_preload<N, G, 1, E, 0, NW>(w, t, tw);
    if constexpr (kUniform) {
        const auto xr = buf_rsrc(x + in_start, valid ? (uint32_t)in_len * ES : 0u);
#pragma unroll
        for (int m = 0; m < E; ++m) u[m] = buf_ld_c((const TIn*)nullptr, xr, (uint32_t)e0 * ES, (uint32_t)(G * m) * ES);
    } else {
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int i = t + G * m;
            u[m] = (valid && i < in_len) ? ld_c(x + in_start + i) : make_float2(0.f, 0.f);
        }
    }
    auto apply_gain = [&] {
        if (a.gain) {   // fused iSTC (rsp_set_prefilter): echo column n times gain[n]
            const auto gr = buf_rsrc(a.gain + in_start, (uint32_t)in_len * 4u);
#pragma unroll
            for (int m = 0; m < E; ++m) u[m] = cscale(u[m], buf_ld_f(gr, (uint32_t)e0 * 4u, (uint32_t)(G * m) * 4u));
        }
    };
    apply_gain();
    float2 hs[kEarly ? E : 1];
    if constexpr (kEarly) {
#pragma unroll
        for (int m = 0; m < E; ++m) hs[m] = buf_ld_f2(hr, (uint32_t)e0 * 8u, (uint32_t)(G * m) * 8u);
    }
    // the FIR segment's staging loads ride on the same memory round trip (a second, dependent
    // round trip made the short rows' FIR phase ~40 % of their lifetime: tools/diag_stamps.py)
    float2 fpre[kUniform ? kFirB : 1];
    if constexpr (kUniform) {
        if (a.do_fir) fir_stage_issue<TIn, G>(fpre, x, a.fir, valid, t, t);
    }
    RSP_STAMP(0, 1, true);
    if (a.do_fir) {
        if (valid)
            for (int z = 0; z < a.nzero; ++z)
                for (int c = a.zero_lo[z] + t; c < a.zero_hi[z]; c += G) st_c<SA>(y + c, make_float2(0.f, 0.f));
        fir_row<TIn, G, SA, WS>(x, y, a.fir, reinterpret_cast<float*>(buf), valid, t, a.gain, st_ok,
                                kUniform ? fpre : nullptr);
    }
    RSP_STAMP(0, 2, false);
    if constexpr (!kDiagPcNoFft) fft_reg_w<N, G, 1, E, 0, NW, WS>(u, buf, t, w);
    RSP_STAMP(0, 3, false);
    if constexpr (kEarly) {
#pragma unroll
        for (int m = 0; m < E; m += 2)   // conj(X.*H), 1/N in H (E is even)
            cmul2_conj(u[m], u[m], hs[m], u[m + 1], u[m + 1], hs[m + 1]);
    } else {
        constexpr int HB = 8;
#pragma unroll
        for (int m0 = 0; m0 < E; m0 += HB) {
            float2 h[HB];   // batches of spectrum loads, then the multiply
#pragma unroll
            for (int m = 0; m < HB; ++m) h[m] = buf_ld_f2(hr, (uint32_t)e0 * 8u, (uint32_t)(G * (m0 + m)) * 8u);
#pragma unroll
            for (int m = 0; m < HB; m += 2)   // conj(X.*H), 1/N in H
                cmul2_conj(u[m0 + m], u[m0 + m], h[m], u[m0 + m + 1], u[m0 + m + 1], h[m + 1]);
        }
    }
    RSP_STAMP(0, 4, false);
    if constexpr (!kDiagPcNoFft) fft_reg_w<N, G, 1, E, 0, NW, WS>(u, buf, t, w);
    RSP_STAMP(0, 5, false);
    if constexpr (kUniform) {
        const auto yr = buf_rsrc(y + out_start, st_ok ? (uint32_t)out_len * 8u : 0u);
#pragma unroll
        for (int m = 0; m < E; ++m) buf_st_f2a<SA>(cconj(u[m]), yr, (uint32_t)e0 * 8u, (uint32_t)(G * m) * 8u);
    } else if (st_ok) {
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int i = t + G * m;
            if (i < out_len) st_c<SA>(y + out_start + i, cconj(u[m]));
        }
    }
    RSP_STAMP(0, 6, false);
    RSP_STAMP(0, 7, true);
    RSP_STAMP_RT(0, 9);
}


// Workgroup size shared by a pair of segment lengths: both run T threads (RPB = T/G rows).
template <int N1, int N2>
struct PairCfg {
    static constexpr int T0 = PcCfg<N1>::G > PcCfg<N2>::G ? PcCfg<N1>::G : PcCfg<N2>::G;
    static constexpr int T = T0 < 256 ? 256 : T0;
    static constexpr int RPB1 = T / PcCfg<N1>::G, RPB2 = T / PcCfg<N2>::G;
    static constexpr size_t L1 = (size_t)RPB1 * PcCfg<N1>::SLOT * sizeof(float2);
    static constexpr size_t L2 = (size_t)RPB2 * PcCfg<N2>::SLOT * sizeof(float2);
    static constexpr size_t lds = L1 > L2 ? L1 : L2;
};

// Single segment (N2 == 0) or two independent segments in one launch: blocks
// [0, nblk2) run segment 2 (the long one, first for a short tail), the rest segment 1.
// `bid` is the block's index among the PC blocks of the launch.
template <typename TIn, int N1, int N2>
__device__ __forceinline__ void pc_mf_block(const TIn* __restrict__ echo, float2* __restrict__ out, const PcMfArgs& a1,
                                            const PcMfArgs& a2, int nblk2, int bid, float2* lds) {
    constexpr int M2 = N2 ? N2 : N1;
    using PC = PairCfg<N1, M2>;
    // unit u of a segment = (row u / nsub, overlap-save sub-block u % nsub)
    // (CPI-to-XCD affinity of the rows was measured in round 5 and rejected:
    //  profiles/r05/affinity/ab_record.txt; the build lives in the history, commit 0cf6ef3)
    if constexpr (N2 != 0) {
        if (bid < nblk2) {
            constexpr int G = PcCfg<N2>::G;
            const int grp = threadIdx.x / G, t = threadIdx.x % G;
            const int ns = a2.nsub > 1 ? a2.nsub : 1;
            const int u = bid * PC::RPB2 + grp;
            pc_row<TIn, N2, G, 0, G == 64>(echo, out, a2, u / ns, t, lds + grp * PcCfg<N2>::SLOT, u % ns);
            return;
        }
    }
    constexpr int G = PcCfg<N1>::G;
    const int grp = threadIdx.x / G, t = threadIdx.x % G;
    const int b = bid - (N2 ? nblk2 : 0);
    const int u = b * PC::RPB1 + grp, ns = a1.nsub > 1 ? a1.nsub : 1;   // (no FIR when ns > 1)
    // a row of one wave (G == 64) synchronises its exchanges within the wave: the rows of a
    // workgroup run independently instead of in barrier lockstep
    pc_row<TIn, N1, G, 0, G == 64>(echo, out, a1, u / ns, t, lds + grp * PcCfg<N1>::SLOT, u % ns);
}

template <typename TIn, int N1, int N2>
__global__ __launch_bounds__((PairCfg<N1, (N2 ? N2 : N1)>::T), RSP_DIAG_PC_WAVES) void pc_mf_kernel(
    const TIn* __restrict__ echo, float2* __restrict__ out, PcMfArgs a1, PcMfArgs a2, int nblk2) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    RSP_STAMP(0, 0, false);
    RSP_STAMP_RT(0, 8);
    pc_mf_block<TIn, N1, N2>(echo, out, a1, a2, nblk2, (int)blockIdx.x, lds);
}


// Dynamic-LDS attribute of a kernel (once per device).
static hipError_t lds_attr(LaunchOnce& once, const void* kernel, size_t lds) {
    return launch_once(once, nullptr, [&](int, int*) {
        return hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    });
}

bool pc_mf_supported(int nfft, int fir_stage_len) {
    switch (nfft) {
        case 64: case 128: case 256: case 512: case 1024: case 2048: case 4096: case 8192:
        case 16384:
            // the FIR stages its input in the row's slot
            return fir_stage_len <= padded_len(nfft);
        default:
            return false;
    }
}

template <typename TIn, int N1, int N2>
static hipError_t launch_pc_mf_n(const TIn* echo, float2* out, const PcMfArgs& a1, const PcMfArgs* a2,
                                 hipStream_t s) {
    constexpr int M2 = N2 ? N2 : N1;
    using PC = PairCfg<N1, M2>;
    static LaunchOnce once;
    constexpr size_t lds = PC::lds + kDiagPcLdsExtra;
    hipError_t e = lds_attr(once, (const void*)pc_mf_kernel<TIn, N1, N2>, lds);
    if (e != hipSuccess) return e;
    const int u1 = a1.rows * (a1.nsub > 1 ? a1.nsub : 1);
    const int nblk1 = (u1 + PC::RPB1 - 1) / PC::RPB1;
    const int u2 = a2 ? a2->rows * (a2->nsub > 1 ? a2->nsub : 1) : 0;
    const int nblk2 = N2 ? (u2 + PC::RPB2 - 1) / PC::RPB2 : 0;
    dim3 grid((unsigned)(nblk1 + nblk2)), block(PC::T);
    hipLaunchKernelGGL((pc_mf_kernel<TIn, N1, N2>), grid, block, lds, s, echo, out, a1, a2 ? *a2 : a1, nblk2);
    return hipGetLastError();
}

#define RSP_PAIR(n1, n2) \
    if (a1.mf.nfft == n1 && a2 && a2->mf.nfft == n2) return launch_pc_mf_n<TIn, n1, n2>(echo, out, a1, a2, s)

template <typename TIn>
static hipError_t launch_pc_mf_t(const TIn* echo, float2* out, const PcMfArgs& a1, const PcMfArgs* a2,
                                 hipStream_t s) {
    // fused pairs of the built-in presets (v2 at 1024..16384 range bins, legacy)
    RSP_PAIR(1024, 1024);
    RSP_PAIR(1024, 4096);
    RSP_PAIR(1024, 8192);
    RSP_PAIR(1024, 16384);
    RSP_PAIR(512, 1024);
    if (a2) return hipErrorNotSupported;
    switch (a1.mf.nfft) {
        case 64: return launch_pc_mf_n<TIn, 64, 0>(echo, out, a1, nullptr, s);
        case 128: return launch_pc_mf_n<TIn, 128, 0>(echo, out, a1, nullptr, s);
        case 256: return launch_pc_mf_n<TIn, 256, 0>(echo, out, a1, nullptr, s);
        case 512: return launch_pc_mf_n<TIn, 512, 0>(echo, out, a1, nullptr, s);
        case 1024: return launch_pc_mf_n<TIn, 1024, 0>(echo, out, a1, nullptr, s);
        case 2048: return launch_pc_mf_n<TIn, 2048, 0>(echo, out, a1, nullptr, s);
        case 4096: return launch_pc_mf_n<TIn, 4096, 0>(echo, out, a1, nullptr, s);
        case 8192: return launch_pc_mf_n<TIn, 8192, 0>(echo, out, a1, nullptr, s);
        case 16384: return launch_pc_mf_n<TIn, 16384, 0>(echo, out, a1, nullptr, s);
        default: return hipErrorInvalidValue;
    }
}
#undef RSP_PAIR

#ifdef RSP_DIAG_STAMPS
}  // namespace rsp
// Dev-only diagnostic export (not in include/rsp.h): copy kernel k's stamps (0 = PC, 1 = MTD)
// of the last launch, kDiagSlots per workgroup, to host.
extern "C" int rsp_diag_stamps(int k, uint64_t* host, int64_t n) {
    if (k < 0 || k > 1 || n < 0 || n > (int64_t)rsp::kDiagWG * rsp::kDiagSlots) return -1;
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(rsp::g_diag), (size_t)n * 8, (size_t)k * rsp::kDiagWG * rsp::kDiagSlots * 8,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -3;
}
namespace rsp {
#endif

bool pc_pair_supported(int n1, int n2) {
    return (n1 == 1024 && (n2 == 1024 || n2 == 4096 || n2 == 8192 || n2 == 16384)) || (n1 == 512 && n2 == 1024);
}

hipError_t launch_pc_mf(const void* echo, int dtype, float2* out, const PcMfArgs& a1, const PcMfArgs* a2,
                        hipStream_t s) {
    if (a1.rows <= 0) return hipSuccess;
    if (dtype == RSP_C64) return launch_pc_mf_t((const float2*)echo, out, a1, a2, s);
    if (dtype == RSP_C32F16) return launch_pc_mf_t((const __half2*)echo, out, a1, a2, s);
    return hipErrorInvalidValue;
}

// ================================================================== CFAR building blocks
// Reference windows of Function_CFAR1D_sub.m:25-28 around cell y of a line whose valid
// part is [lo, hi): left = [y-save-ref, y-save-1], right = [y+save+1, y+save+ref]; a side
// that leaves [lo, hi) is replaced by the other side's mean (:30-39).  Window sums are
// precomputed as direct left-to-right sums of `ref` cells (the order mean() adds them),
// so a cell needs two sum lookups.  max/min of the two means = max/min of the two sums
// divided once (division by a positive constant is monotonic in IEEE arithmetic).
__device__ __forceinline__ uint8_t cfar_test(float x, float sl, float sr, bool lok, bool rok, int method, float Tr) {
    // fp32 threshold max|min(sum_L, sum_R) * (T/ref); the fp64 reference computes
    // (sum/ref)*T -- the two differ by ~1 ulp, far inside the near-threshold band
    const float a = lok ? sl : sr;
    const float b = rok ? sr : sl;
    return x >= (method == 0 ? fmaxf(a, b) : fminf(a, b)) * Tr ? 1 : 0;
}

__device__ __forceinline__ bool in_segs(int c, int nseg, const int* lo, const int* hi) {
    bool in = false;
#pragma unroll
    for (int s = 0; s < RSP_MAX_SEG; ++s)
        if (s < nseg) in |= (c >= lo[s] && c < hi[s]);
    return in;
}

__device__ __forceinline__ void seg_of(int c, int nseg, const int* lo, const int* hi, int& slo, int& shi) {
    slo = 0;
    shi = 0;
#pragma unroll
    for (int s = 0; s < RSP_MAX_SEG; ++s)
        if (s < nseg && c >= lo[s] && c < hi[s]) {
            slo = lo[s];
            shi = hi[s];
        }
}

// Doppler CFAR over a column-major tile in LDS: column c = mag[c*ms + v], v < V (zero band
// already applied).  Thread (c, g) owns rows [v0, v1); sums[c*ms + a] must hold the window
// sums for every a with a + ref <= V.  Writes flags to out[v*R] (out already offset by r).
__device__ __forceinline__ void doppler_sums(const float* mag, float* sums, int V, int ref, int v0, int v1) {
    for (int a = v0; a < v1; ++a) {
        if (a + ref > V) break;
        float s = 0.f;
        for (int k = 0; k < ref; ++k) s += mag[a + k];
        sums[a] = s;
    }
}

__device__ __forceinline__ uint8_t doppler_test(const float* mag, const float* sums, const CfarVArgs& cv,
                                                bool col_on, int v) {
    uint8_t f = 0;
    if (col_on && v >= cv.lo && v < cv.hi) {
        const int l1 = v - cv.save - cv.ref, r1 = v + cv.save + 1;
        const bool lok = l1 >= cv.lo, rok = r1 + cv.ref <= cv.hi;
        f = cfar_test(mag[v], lok ? sums[l1] : 0.f, rok ? sums[r1] : 0.f, lok, rok, cv.method, cv.Tr);
    }
    return f;
}

__device__ __forceinline__ void doppler_flags(const float* mag, const float* sums, const CfarVArgs& cv, bool col_on,
                                              int v0, int v1, uint8_t* __restrict__ out, size_t R, bool rv) {
    out += (size_t)v0 * R;
    for (int v = v0; v < v1; ++v) {
        const uint8_t f = doppler_test(mag, sums, cv, col_on, v);
        if (rv) *out = f;
        out += R;
    }
}

// ================================================================== MTD (+ Doppler CFAR)
// One workgroup = W range bins x all P pulses.  Thread (c, g): range bin c of the tile,
// pulses g + G*m (m < E) -- the strided pattern of fft_reg, so the pulse-compressed
// samples load straight into registers with W-wide coalesced rows, the slow-time FFT
// runs register-resident with LDS exchanges, and |X| leaves in coalesced RDM rows.
template <int P, int BEAMS = 1>
struct MtdCfg {
    // elements per thread: 16 (24 for the 3*2^k lengths); from P = 512 on (one beam) the
    // workgroup grows with G (512..1024 threads) so a tile keeps >= 8..16 range bins
    // (>= 64..128-B row segments) and a thread still holds 16 elements -- E = 32 at 256 threads
    // needed 169 VGPRs, 2 waves per SIMD
    static constexpr int E = (P % 3 == 0) ? 24 : 16;
    static constexpr int G = P / E;                    // threads per range bin
    // threads per workgroup (512 for P = 256 measured neutral at c4: 529 vs 523 us per launch)
    static constexpr int T = (BEAMS == 1 && P >= 512 && P % 3 != 0) ? (G * 16 < 1024 ? G * 16 : 1024) : kBlock;
    // minimum waves per SIMD (__launch_bounds__' second argument): two 512-thread workgroups
    // per CU need <= 128 VGPRs
    static constexpr int WPE = T == 512 ? 4 : 1;
    static constexpr int W = T / G;                    // range bins per workgroup
    static constexpr int SLOT = padded_len(P);         // FFT exchange slot (float2)
    static constexpr int MS = P + 1;                   // odd float stride of a CFAR column
    static constexpr int SPAD = 32;                    // sums pad: save + ref + 2 <= 32 (host-checked)
    static constexpr int SMS = P + 2 * SPAD + 1;       // padded sums column (odd stride)
    static constexpr size_t lds_fft = (size_t)W * SLOT * sizeof(float2);
    static constexpr size_t lds_cfar = (size_t)W * (MS + SMS) * sizeof(float);
    static constexpr size_t lds = lds_fft > lds_cfar ? lds_fft : lds_cfar;
    // REF > 0: the window sums stay in registers; LDS holds only a padded magnitude column
    // (SPAD pad cells on each side, odd stride), inside the FFT exchange area
    static constexpr int MS2 = P + 2 * SPAD + 1;
    static constexpr size_t lds_cfar_reg = (size_t)W * MS2 * sizeof(float);
    static constexpr size_t lds_reg = lds_fft > lds_cfar_reg ? lds_fft : lds_cfar_reg;
    template <int REF>
    static constexpr size_t lds_for() { return REF > 0 ? lds_reg : lds; }
    static_assert(G * E == P && (G & (G - 1)) == 0 && G <= T, "MTD tiling");
};

// Per-row outputs of the Doppler CFAR at cell (v, r) of launch CPI `cpi`: flagV (if requested),
// the flag plane's background (flagV when the range stage is off, else 0) and, for a hit
// with the range stage on, an entry in the hit list (one atomic per wave and row).
struct DopplerOut {
    __amdgpu_buffer_rsrc_t fv, fl;   // flagV / flag planes of this CPI (num_records 0 if absent)
    uint32_t vo;                     // this lane's cell offset (row v0, column r) or kOob
    uint32_t R;
    uint32_t* hits;                  // this workgroup's region of the hit list
    uint32_t* lds_count;             // workgroup hit counter (LDS)
    uint32_t cell0;                  // linear index of (v0, r) within the launch
    bool want_fv, fused, rflag;
    bool coherent;                   // hit entries consumed inside this launch (fused chain):
                                     // agent-scope stores; else plain stores (consumed by a
                                     // later launch -- an sc1 store writes through the L2)
    bool zero_bg;                    // rflag: write the flag plane's zero background here
};

// The Doppler-stage outputs of a thread's run of N rows (bit i of `mask` = row v0+i is a hit);
// called with every lane of the wave active (its ballots and prefix-sum shuffles read all lanes):
// flagV / flag bytes where requested (uniform branches, once per run), and the hits appended to
// the workgroup's list.  Hits are sparse, so the append path is entered only by waves that
// have one: one ballot over the masks, then per row one ballot and one LDS atomic per wave.
template <int N, typename Hit>
__device__ __forceinline__ void doppler_emit(const DopplerOut& o, bool anyhit, const Hit& hit) {
    if (o.want_fv) {
#pragma unroll
        for (int i = 0; i < N; ++i) buf_st_u8(hit(i) ? 1u : 0u, o.fv, o.vo, (uint32_t)i * o.R);
    }
    if (!o.fused) return;
    if (!o.rflag) {   // flag = flagV (executeCFAR.m:91)
#pragma unroll
        for (int i = 0; i < N; ++i) buf_st_u8(hit(i) ? 1u : 0u, o.fl, o.vo, (uint32_t)i * o.R);
        return;
    }
    if (o.zero_bg) {   // zero background (here, or pre-zeroed); the range stage sets the detections
#pragma unroll
        for (int i = 0; i < N; ++i) buf_st_u8(0, o.fl, o.vo, (uint32_t)i * o.R);
    }
    if (__ballot(anyhit) == 0) return;   // the common case: no hit in the wave's rows
    // row by row: one ballot per row of the run gives the row's hit lanes, so the wave's
    // entries go out row-major -- each store instruction writes the row's hits as one
    // contiguous run (a lane-major run per lane made every store a scatter), and neighbouring
    // entries are neighbouring columns of one row, whose range windows overlap.  The
    // counts are scalar (popcounts of the ballots, each taken once): one LDS atomic per wave,
    // its result broadcast by readfirstlane (no shuffle through LDS).
    uint64_t bal[N];
    uint32_t total = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        bal[i] = __ballot(hit(i));
        total += (uint32_t)__popcll(bal[i]);
    }
    uint32_t base = 0;
    if (__lane_id() == 0) base = atomicAdd(o.lds_count, total);
    base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const uint64_t b = bal[i];
        if (b == 0) continue;   // (wave-uniform)
        if (hit(i)) {
            const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
            uint32_t* dst = o.hits + base + below;
            if (o.coherent) st_u32_sc1(dst, o.cell0 + (uint32_t)i * o.R);
            else *dst = o.cell0 + (uint32_t)i * o.R;
        }
        base += (uint32_t)__popcll(b);
    }
}

// the same for a row bit mask (bit i = row v0+i is a hit)
template <int N>
__device__ __forceinline__ void doppler_emit_mask(const DopplerOut& o, uint32_t mask) {
    doppler_emit<N>(o, mask != 0u, [&](int i) { return ((mask >> i) & 1u) != 0u; });
}

template <int N>
__device__ __forceinline__ void doppler_flags(const float* mag, const float* sums, const CfarVArgs& cv, bool col_on,
                                              int v0, int v1, const DopplerOut& o) {
    uint32_t mask = 0;
#pragma unroll
    for (int i = 0; i < N; ++i)
        if (v0 + i < v1 && doppler_test(mag, sums, cv, col_on, v0 + i)) mask |= 1u << i;
    doppler_emit_mask<N>(o, mask);
}

// Doppler CFAR with the reference's window compiled in (REF = 5 reference and SAVE = 7 guard
// cells, main_cfar.m:40-58; other windows take the runtime path; the method and the row band
// stay runtime).  A thread owns a run of E rows of one range column: it reads its rows and the
// (left, right) window cells of every row as pairs from the padded magnitude column -- the two
// cells of a pair lie 2 SAVE + REF + 1 apart, one ds_read2 into a register pair -- and forms each
// row's two window sums together with packed adds (each sum still the left-to-right add of its
// REF cells, mean()'s order), in registers: no sums array, no second barrier, and the LDS
// footprint stays inside the FFT exchange area.
template <int P, int REF, int BEAMS>
__device__ __forceinline__ void doppler_cfar_fixed(const float* mag, const CfarVArgs& cv, bool col_on, int v0,
                                                   const DopplerOut& o) {
    static_assert(REF == 5, "the compiled-in window is the reference's (5 reference, 7 guard cells)");
    constexpr int SAVE = 7;
    // mag: this column's magnitudes, mag[v] for v in [-SPAD, P + SPAD) (pad cells unused:
    // every row in [lo, hi) has at least one window inside the column, the other is selected
    // away).  The left window of row v0+i starts at v0+i-SAVE-REF, the right one at
    // v0+i+SAVE+1.
    constexpr int E = MtdCfg<P, BEAMS>::E, NL = E + REF - 1, DLR = 2 * SAVE + REF + 1;
    const float* bl = mag + v0 - SAVE - REF;
    v2f lr[NL];   // (left cell, right cell) of window position i: bl[i], bl[i + DLR]
    float m[E];   // the cells under test, bl[SAVE + REF + i]: inside the pairs' span
    if constexpr (NL == 20 && DLR == 20) {
        // one asm block: 20 ds_read2_b32 straight into the pairs (hipcc merges neighbouring
        // cells instead and spends ~40 v_mov re-pairing them), and the wait on them
        const uint32_t ad = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)bl;
#define RSP_PAIR_LD(i, j) "ds_read2_b32 %" #i ", %20 offset0:" #i " offset1:" #j "\n\t"
        asm volatile(RSP_PAIR_LD(0, 20) RSP_PAIR_LD(1, 21) RSP_PAIR_LD(2, 22) RSP_PAIR_LD(3, 23) RSP_PAIR_LD(4, 24)
                     RSP_PAIR_LD(5, 25) RSP_PAIR_LD(6, 26) RSP_PAIR_LD(7, 27) RSP_PAIR_LD(8, 28) RSP_PAIR_LD(9, 29)
                     RSP_PAIR_LD(10, 30) RSP_PAIR_LD(11, 31) RSP_PAIR_LD(12, 32) RSP_PAIR_LD(13, 33)
                     RSP_PAIR_LD(14, 34) RSP_PAIR_LD(15, 35) RSP_PAIR_LD(16, 36) RSP_PAIR_LD(17, 37)
                     RSP_PAIR_LD(18, 38) RSP_PAIR_LD(19, 39) "s_waitcnt lgkmcnt(0)"
                     : "=&v"(lr[0]), "=&v"(lr[1]), "=&v"(lr[2]), "=&v"(lr[3]), "=&v"(lr[4]), "=&v"(lr[5]), "=&v"(lr[6]),
                       "=&v"(lr[7]), "=&v"(lr[8]), "=&v"(lr[9]), "=&v"(lr[10]), "=&v"(lr[11]), "=&v"(lr[12]),
                       "=&v"(lr[13]), "=&v"(lr[14]), "=&v"(lr[15]), "=&v"(lr[16]), "=&v"(lr[17]), "=&v"(lr[18]),
                       "=&v"(lr[19])
                     : "v"(ad)
                     : "memory");
#undef RSP_PAIR_LD
#pragma unroll
        for (int i = 0; i < E; ++i) m[i] = SAVE + REF + i < NL ? lr[SAVE + REF + i].x : lr[SAVE + REF + i - DLR].y;
    } else {
#pragma unroll
        for (int i = 0; i < NL; ++i) lr[i] = (v2f){bl[i], bl[i + DLR]};
#pragma unroll
        for (int i = 0; i < E; ++i) m[i] = bl[SAVE + REF + i];
    }
    const int kl = cv.lo + SAVE + REF - v0;     // row v0+i has a left window iff i >= kl
    const int kr = cv.hi - SAVE - 1 - REF - v0; // ... and a right window iff i <= kr
    const int b0 = cv.lo - v0, b1 = cv.hi - v0; // tested rows: b0 <= i < b1
    const bool go = cv.method == 0;
    // per-row hit predicates (lane masks, not a packed bit mask: each row's ballot is then the
    // compare's own result, with no bit packing and extraction around it)
    bool h[E];
    if (kl <= 0 && kr >= E - 1 && b0 <= 0 && b1 >= E && go) {
        // the common case: every row of the run is tested and has both windows (GO): the same
        // sums, the greater of the two (magnitude sums are never NaN or -0, so max is the
        // compare-select), without the per-row window and band selects
#pragma unroll
        for (int i = 0; i < E; ++i) {
            v2f sw = lr[i];
#pragma unroll
            for (int q = 1; q < REF; ++q) sw += lr[i + q];
            h[i] = col_on & (m[i] >= __builtin_fmaxf(sw.x, sw.y) * cv.Tr);
        }
    } else {
#pragma unroll
        for (int i = 0; i < E; ++i) {
            v2f sw = lr[i];
#pragma unroll
            for (int q = 1; q < REF; ++q) sw += lr[i + q];
            const float sl = sw.x, sr = sw.y;
            const bool lok = i >= kl, rok = i <= kr;
            const float x = lok ? sl : sr, y = rok ? sr : sl;   // one-sided fallback (:30-39)
            const float th = (go ? __builtin_fmaxf(x, y) : __builtin_fminf(x, y)) * cv.Tr;
            h[i] = col_on & (i >= b0) & (i < b1) & (m[i] >= th);
        }
    }
    bool any = false;
#pragma unroll
    for (int i = 0; i < E; ++i) any |= h[i];
    // (outside the divergent branches: the emission's ballots need every lane)
    doppler_emit<E>(o, any, [&](int i) { return h[i]; });
}

// The run of Doppler rows a CFAR thread takes: runs 0 and G-1 (the only ones near the column's
// ends with the reference's full row band, whose windows need the one-sided selects) go to the
// first wave's threads, so one wave of the workgroup runs the edge path instead of two.
template <int G, int W>
__device__ __forceinline__ int cfar_run(int g) {
    if constexpr (64 % W == 0 && 64 / W >= 2 && G > 2) return g == 0 ? 0 : (g == 1 ? G - 1 : g - 1);
    else return g;
}

// Threads first, first + step, ... evaluate the hits of region rg: REF/SAVE > 0 compile-time
// windows (every load of a hit's window issues at once); 0: the runtime ref/save of CfarRArgs.
template <int REF, int SAVE, int LA = 0>
__device__ __forceinline__ void cfar_hit_region(const float* __restrict__ rdm, uint8_t* __restrict__ flag,
                                                const uint32_t* __restrict__ hits,
                                                const uint32_t* __restrict__ counts, int rg, int region,
                                                const CfarRArgs& a, int first, int step = 64) {
    const uint32_t n = ld_u32<LA>(counts + rg);
    const uint32_t* list = hits + (size_t)rg * region;
    const int R = a.R, V = a.V;
    const int ref = REF > 0 ? REF : a.ref, save = REF > 0 ? SAVE : a.save;
    for (uint32_t i = first; i < n; i += step) {
        const uint32_t idx = ld_u32<LA>(list + i);
        const uint32_t row = idx / (uint32_t)R;        // cpi * V + v
        const int r = (int)(idx - row * (uint32_t)R);
        const int v = (int)(row % (uint32_t)V);
        int slo, shi;
        seg_of(r, a.nseg, a.seg_lo, a.seg_hi, slo, shi);
        if (shi <= slo) continue;
        const bool zrow = v >= a.cz_lo && v < a.cz_hi;
        const float* xr = rdm + (size_t)row * R;
        auto X = [&](int c) { return (!zrow && c >= 0 && c < R) ? ld_f<LA>(xr + c) : 0.f; };
        int best = -1;
        float bx = 0.f;
#pragma unroll
        for (int e = -1; e <= 1; ++e) {
            const int q = r + e;
            float sl = 0.f, sr = 0.f;
            if constexpr (REF > 0) {
#pragma unroll
                for (int k = 0; k < REF; ++k) {
                    sl += X(q - SAVE - REF + k);
                    sr += X(q + SAVE + 1 + k);
                }
            } else {
                for (int k = 0; k < ref; ++k) {
                    sl += X(q - save - ref + k);
                    sr += X(q + save + 1 + k);
                }
            }
            const bool lok = q - save - ref >= slo, rok = q + save + ref < shi;
            const float xq = X(q);
            if (q >= slo && q < shi && cfar_test(xq, sl, sr, lok, rok, a.method, a.Tr) && (best < 0 || xq > bx)) {
                best = q;
                bx = xq;
            }
        }
        if (best >= 0) flag[(size_t)row * R + best] = 1;
    }
}

// The previous chunk's range stage inside an MTD launch: workgroup wg of the launch's nwg
// evaluates the hit regions wg, wg + nwg, ... of the previous chunk on this pipeline (the same
// tile shape, so normally exactly one), all its threads sharing a region's hits.  `skip`: the
// region-wg hits already done by a RangeJob.
__device__ __forceinline__ void prev_chunk_hits(const MtdArgs& a, int wg, int nwg, int skip) {
    const bool ref57 = a.prev_cr.ref == 5 && a.prev_cr.save == 7;
    for (int rg = wg; rg < a.prev_nregions; rg += nwg) {
        const int first = (int)threadIdx.x + (rg == wg ? skip : 0);
        if (ref57)
            cfar_hit_region<5, 7>(a.prev_rdm, a.prev_flag, a.prev_hits, a.prev_count, rg, a.prev_region, a.prev_cr,
                                  first, blockDim.x);
        else
            cfar_hit_region<0, 0>(a.prev_rdm, a.prev_flag, a.prev_hits, a.prev_count, rg, a.prev_region, a.prev_cr,
                                  first, blockDim.x);
    }
}

// The range-stage share of one MTD workgroup for the reference's window (5 reference + 7 guard
// cells, executeCFAR.m:45-84 with Function_CFAR1D_sub_fixCells.m:34-58): its region's first
// blockDim hits, one per thread.  The hit count and the thread's hit index are loaded before
// the tile, the 17 RDM cells of the hit's row that the test reads (r-13 .. r-7, r-1 .. r+1,
// r+7 .. r+13) right after the tile's own loads,
// and the test + first-maximum scatter run after the tile -- the three dependent gathers hide
// under the tile's FFT and Doppler CFAR instead of trailing the workgroup.
// The thread's index in its workgroup.  OPQ: through an empty volatile asm, so the value (and
// everything derived from it) is recomputed where it is used instead of being hoisted out of the
// dataflow kernel's item loop and held -- spilled -- across every item.
template <bool OPQ>
__device__ __forceinline__ int tid_of() {
    int t = (int)threadIdx.x;
    if constexpr (OPQ) asm volatile("" : "+v"(t));
    return t;
}

// Where a range job reads and writes: the previous chunk's RDM / flag planes, hit lists and
// counts (MtdArgs::prev_* in the chunked pipeline; the dataflow kernel's ring slots otherwise).
struct RangeSrc {
    const float* rdm;
    uint8_t* flag;
    const uint32_t* hits;
    const uint32_t* count;
    int region;
    const CfarRArgs& cr;
    __device__ __forceinline__ static RangeSrc of(const MtdArgs& a) {
        return RangeSrc{a.prev_rdm, a.prev_flag, a.prev_hits, a.prev_count, a.prev_region, a.prev_cr};
    }
};

// LA: cache policy of the job's loads (kSc1 when the hit lists and the RDM were written by other
// workgroups of the same launch).
template <int LA = 0>
struct RangeJob57T {
    // the cells executeCFAR's fixCells test of r-1, r, r+1 reads (5 reference cells beyond 7 guard
    // cells on each side): r-13 .. r-7, r-1 .. r+1, r+7 .. r+13
    static constexpr int NX = 17;
    static constexpr int kLoads = NX;   // fetch_cells' gathers (the hook of mtd_tile)
    static __device__ __forceinline__ constexpr int cell_off(int k) { return k < 7 ? k - 13 : (k < 10 ? k - 8 : k - 3); }
    // the NX cells of hit column r in row `row` (range-checked: zero outside [0, R), on a
    // zeroed row or for a lane without a hit), issued as one batch
    static __device__ __forceinline__ void gather(float (&x)[NX], __amdgpu_buffer_rsrc_t rr, uint32_t row, int r,
                                                  bool live, int R) {
        const uint32_t rowoff = row * (uint32_t)R;
        const uint32_t rlive = live ? (uint32_t)R : 0u;   // q in [0, R) of a live lane: one unsigned compare
#pragma unroll
        for (int k = 0; k < NX; ++k) {
            const int q = r + cell_off(k);
            x[k] = buf_ld_fa<LA>(rr, (uint32_t)q < rlive ? (rowoff + (uint32_t)q) * 4u : kOob, 0u);
        }
    }
    // executeCFAR.m:45-84 at hit column r: the fixCells test of r-1, r, r+1 (one-sided windows
    // at the segment edges) and the first maximum among the passing cells, or -1
    static __device__ __forceinline__ int test(const float (&x)[NX], int r, int slo, int shi, const CfarRArgs& c) {
        int best = -1;
        float bx = 0.f;
#pragma unroll
        for (int e = -1; e <= 1; ++e) {
            const int q = r + e;   // left window q-12 .. q-8 = x[e+1 ..], centre x[8+e], right q+8 .. q+12
            float sl = 0.f, sr = 0.f;
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                sl += x[e + 1 + k];
                sr += x[11 + e + k];
            }
            const bool lok = q - 12 >= slo, rok = q + 12 < shi;
            const float xq = x[8 + e];
            if (q >= slo && q < shi && cfar_test(xq, sl, sr, lok, rok, c.method, c.Tr) && (best < 0 || xq > bx)) {
                best = q;
                bx = xq;
            }
        }
        return best;
    }
    uint32_t n = 0, idx = 0;
    float x[NX];
    __device__ __forceinline__ void fetch_idx(const RangeSrc& s, int rg) {
        // both loads issue at once: a region holds W*P >= blockDim entries, so the index load
        // is in bounds (and ignored) past the count -- no count -> index round trip
        n = ld_u32<LA>(s.count + rg);
        idx = ld_u32<LA>(s.hits + (size_t)rg * s.region + tid_of<LA != 0>());
    }
    __device__ __forceinline__ void fetch_cells(const RangeSrc& s) {
        // Every wave of every MTD workgroup issues these 17 loads, unconditionally: a lane
        // without a cell (no hit, no job) loads through the buffer range check (voffset kOob:
        // 0, no memory access).  A branch around them would leave the waits of the tile's FFT
        // (vmcnt counts in issue order) merged from two paths, so a wave with hits would wait
        // for its gathers before its first butterfly (c3: 3.8 us per 16-CPI launch).
        const CfarRArgs& c = s.cr;
        const bool mine = (uint32_t)tid_of<LA != 0>() < n;
        const uint32_t R = c.R > 0 ? (uint32_t)c.R : 1u, V = c.V > 0 ? (uint32_t)c.V : 1u;   // (no job: unset)
        const uint32_t row = idx / R;
        const int r = (int)(idx - row * R);
        const int v = (int)(row % V);
        const bool zrow = v >= c.cz_lo && v < c.cz_hi;
        gather(x, buf_rsrc(s.rdm, kOob), row, r, mine && !zrow, c.R);   // (job => the RDM is < kOob bytes)
    }
    __device__ __forceinline__ void finish(const RangeSrc& s) {
        if ((uint32_t)tid_of<LA != 0>() >= n) return;
        const CfarRArgs& c = s.cr;
        const uint32_t row = idx / (uint32_t)c.R;
        const int r = (int)(idx - row * (uint32_t)c.R);
        int slo, shi;
        seg_of(r, c.nseg, c.seg_lo, c.seg_hi, slo, shi);
        if (shi <= slo) return;
        const int best = test(x, r, slo, shi, c);
        if (best >= 0) s.flag[(size_t)row * c.R + best] = 1;
    }
};
using RangeJob57 = RangeJob57T<0>;

template <int LA = 0>
struct RangeHookT {   // mtd_tile's after_loads(): the range job's gathers (a workgroup without a
                      // job, rj.n == 0, issues them with every lane out of range)
    RangeJob57T<LA>& rj;
    const RangeSrc& s;
    static constexpr int kLoads = RangeJob57T<LA>::kLoads;
    __device__ __forceinline__ void operator()() const { rj.fetch_cells(s); }
};

struct NoHook {
    static constexpr int kLoads = 0;   // vector-memory operations operator() issues
    __device__ __forceinline__ void operator()() const {}
};

// MTD tile loads by LDS-DMA (round 4; A/B in profiles/r04/ab/: c4 +5.8 %,
// c3 +1.5 %, c5 +0.4 %, outputs bit-identical): one beam, no MTI, default cache policy.  The
// tile's P rows of W complex columns (W*8 bytes each) go to LDS as 16-byte pieces
// (buffer_load_dwordx4 ... lds, no VGPR destination); a wave instruction covers 64/(W/2) whole
// rows; a row past pin loads 0 through the range check.  The range job's gathers issue behind the
// pieces and stay in flight across the barrier.  -DRSP_MTD_NO_DMA (dev-only) restores register
// loads for A/B runs.
template <int P, int BEAMS, int LA, int W>
__host__ __device__ constexpr bool kMtdDma() {
#ifndef RSP_MTD_NO_DMA
    // (LA = kSc1, the dataflow kernel: the pieces are sc1 LDS-DMA loads, L1 bypassed like its
    // register loads)
    return BEAMS == 1 && (LA == 0 || LA == kSc1) && W >= 2 && W <= 128 && 64 % (W / 2) == 0;
#else
    return false;
#endif
}
template <int P, int W, int T, int LA = 0>
__device__ __forceinline__ void mtd_dma_issue(__amdgpu_buffer_rsrc_t src, uint32_t col0, uint32_t R, unsigned char* smem,
                                              int tx) {
    constexpr int LPR = W / 2;                    // lanes per row (16 B = 2 columns each)
    constexpr int BYTES = P * W * 8;
    constexpr int NQ = BYTES / (T * 16);          // DMA instructions per thread
    static_assert(BYTES % (T * 16) == 0 && 64 % LPR == 0, "MTD DMA tiling");
    const int t = tx;
    const int wb = __builtin_amdgcn_readfirstlane(t & ~63);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int piece = q * T + t;              // 16-byte piece of the linear [P][W] image
        const int row = piece / LPR, cp = (piece % LPR) * 2;
        // (no per-lane range test: a column past R_out of a right-edge tile reads the next
        // row's first samples -- or 0 past the plane -- into an LDS column whose thread has
        // rv == false, so nothing computed from it is stored; a select here made hipcc split
        // every DMA into two exec-masked copies)
        const uint32_t vo = ((uint32_t)row * R + col0 + (uint32_t)cp) * 8u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(src, (lds_void*)(smem + (q * T + wb) * 16), 16, vo, 0, 0, LA);
    }
}

// MTD: one workgroup = W range bins x all P pulses.  Thread (c, g): range bin c of the
// tile, pulses g + G*m (m < E) -- the strided pattern of fft_reg, so the pulse-compressed
// samples load straight into registers with W-wide coalesced rows, the slow-time FFT runs
// register-resident with LDS exchanges, and |X| leaves in coalesced RDM rows.  The fftshift
// offset is 0 or P/2, a multiple of G, so bin g + G*m lands in row g + G*((m + shift/G) mod E):
// a wave-uniform rotation, and every row offset is an SGPR operand of the buffer access.
// REF > 0: Doppler CFAR specialised on the reference window; REF == 0: runtime window.
// P is the Doppler FFT length; a CPI supplies a.pin <= P pulses per beam (rows past pin are
// the zero padding of fft(x, P, 1): out of the buffer's range, they load as 0).  BEAMS == 2:
// the DMX pair -- both beams' slow-time FFTs, RDM = |X_0| + |X_1|, diff = |X_1| - |X_0|.
// Pointers of one MTD work item: the CPI's planes and the tile's hit-list region.
struct MtdTile {
    const float2* pc;      // the CPI's first PC row (beam 0); beam b starts pin rows later
    float* rdm;            // the CPI's RDM plane
    float* diff;           // the CPI's DMX difference plane, or null
    uint8_t* flagV;        // the CPI's flagV plane, or null
    uint8_t* flag;         // the CPI's flag plane, or null (no CFAR)
    uint32_t* hits;        // this tile's hit-list region (W*P entries), or null
    uint32_t* hit_count;   // where the tile's hit count goes
    uint32_t cell_base;    // hit-list number of the CPI's cell (0, 0)
    int bx;                // tile index along range
};

// fn(mm) for the thread's rows g + G*mm (mm < E) inside [lo, hi) (G a power of two; the
// arithmetic shift floors, so (x + G - 1) >> log2(G) is ceil(x / G) for negative x too)
template <int G, int E, typename F>
__device__ __forceinline__ void own_rows(int g, int lo, int hi, const F& fn) {
    constexpr int LG = __builtin_ctz(G);
    static_assert((G & (G - 1)) == 0, "G is a power of two");
    const int a0 = max(0, (lo - g + G - 1) >> LG), b0 = min(E, (hi - g + G - 1) >> LG);
#pragma clang loop unroll(disable) vectorize(disable)
    for (int mm = a0; mm < b0; ++mm) fn(mm);
}

// MTD load-phase wave priority (round 4, profiles/r04/ab/session11_mtd_prio.txt): for Doppler
// lengths P >= 256 a tile's waves run at priority 3 until the tile's loads are issued (mtd_block
// raises it, mtd_tile drops it before the FFT), so a newly resident workgroup gets its loads out
// ahead of the other tiles' compute: c4 MTD 690-707 -> 658-663 us, c4 +3.5 %, outputs identical.
// At P = 128 (c3) the same cost 1-2 %, and in the PC kernel 10 % (its rows' compute is the long
// phase), so neither has it.
#ifndef RSP_MTD_PRIO
#define RSP_MTD_PRIO 3      // (dev-only -D for A/B)
#endif
#ifndef RSP_MTD_PRIO_MINP
#define RSP_MTD_PRIO_MINP 256
#endif
constexpr int kMtdLoadPrio = RSP_MTD_PRIO, kMtdLoadPrioMinP = RSP_MTD_PRIO_MINP;

// One MTD tile: W range bins x all P pulses.  LA / SA: cache policy of the PC loads and of
// the RDM stores (kSc1 when another workgroup of the same launch consumes them).
// after_loads(): called once the tile's first-beam loads are issued (RangeJob57 gathers).
template <int P, int REF, int BEAMS, int LA, int SA, typename Hook = NoHook, bool OPQ = false>
__device__ __forceinline__ void mtd_tile(const MtdTile& T, const MtdArgs& a, unsigned char* smem, uint32_t* s_hits,
                                         const Hook& after_loads = Hook()) {
    using C = MtdCfg<P, BEAMS>;
    constexpr int G = C::G, E = C::E, W = C::W;
    const int tx = tid_of<OPQ>();
    if (tx == 0) *s_hits = 0u;   // published by the FFT's barriers
    const int c = tx % W, g = tx / W;
    const uint32_t R = (uint32_t)a.R_out;
    const int r = T.bx * W + c;
    const bool rv = r < (int)R;
    const uint32_t plane = (uint32_t)P * R;                     // output plane (P Doppler rows)
    const uint32_t cell = (uint32_t)g * R + (uint32_t)r;        // element (g, r) of a plane
    const int pin = a.pin;
    const uint32_t vo_in = rv ? cell * 8u : kOob;
    float2 u[E];
    float m0[BEAMS == 2 ? E : 1];     // |X_0| while beam 1 runs
    // the FFT's twiddles are loaded up front, with the tile: a twiddle load issued later (inside
    // the FFT) would make every wait for it also wait for the after_loads() gathers (vmcnt
    // counts in issue order)
    constexpr int NW = tw_regs<P, E>() > 0 ? tw_regs<P, E>() : 1;
    float2 tw[NW];
    tw_preload<P, G, 1, E, 0, NW>(tw, g, a.tw);
#pragma unroll
    for (int b = 0; b < BEAMS; ++b) {
        const auto src = buf_rsrc(T.pc + (size_t)b * pin * R, (uint32_t)pin * R * 8u);
        if (a.mti_lag > 0) {   // fused MTI (wave-uniform): pulse p = PC(p + lag) - PC(p), 0 past pin - lag
            const int lag = a.mti_lag;
#pragma unroll
            for (int m = 0; m < E; ++m) {
                const float2 v0 = buf_ld_f2a<LA>(src, vo_in, (uint32_t)(G * m) * R * 8u);
                const float2 v1 = buf_ld_f2a<LA>(src, vo_in, (uint32_t)(G * m + lag) * R * 8u);
                const float w = g + G * m + lag < pin ? a.win[g + G * m] : 0.f;
                u[m] = make_float2((v1.x - v0.x) * w, (v1.y - v0.y) * w);
            }
        } else if constexpr (kMtdDma<P, BEAMS, LA, W>()) {
            // the tile's P rows x W columns land in LDS by DMA (row-major [p][c], linear), then
            // thread (c, g) reads its strided pulses; the range job's gathers issue behind the
            // DMA and stay in flight across the barrier (a counted vmcnt, a raw s_barrier)
            float wv[E];
#pragma unroll
            for (int m = 0; m < E; ++m) wv[m] = a.win[g + G * m];
            mtd_dma_issue<P, W, C::T, LA>(src, (uint32_t)(T.bx * W), R, smem, tx);
            // (a compiler barrier: the range gathers below must issue after every DMA piece, or
            // the counted vmcnt would not cover the pieces -- hipcc interleaved them otherwise)
            asm volatile("" ::: "memory");
            // (one path per kernel instance -- the range job is a template choice, not a runtime
            // branch: where a job / no-job branch merged, hipcc's waitcnt pass, which cannot read
            // an asm wait, counted from the no-job side and made the window multiply wait for
            // most gathers).  The weights and twiddles are older than the gathers, so the wait
            // covers them; redefined behind it, no later use of them waits for the gathers, which
            // stay in flight through the FFT and the Doppler CFAR (lds_barrier).
            after_loads();
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(Hook::kLoads) : "memory");
#pragma unroll
            for (int m = 0; m < E; ++m) asm volatile("" : "+v"(wv[m]));
#pragma unroll
            for (int i = 0; i < NW; ++i) asm volatile("" : "+v"(tw[i]));
            // (the barrier as asm with a memory clobber: __builtin_amdgcn_s_barrier touches no
            // memory at the IR level, so nothing would keep the LDS reads below it)
            asm volatile("s_barrier" ::: "memory");
            const float2* l = reinterpret_cast<const float2*>(smem);
#pragma unroll
            for (int m = 0; m < E; ++m) {
                const float2 v = l[(g + G * m) * W + c];
                u[m] = make_float2(v.x * wv[m], v.y * wv[m]);
            }
        } else {
#pragma unroll
            for (int m = 0; m < E; ++m) {
                const float2 v = buf_ld_f2a<LA>(src, vo_in, (uint32_t)(G * m) * R * 8u);
                const float w = a.win[g + G * m];
                u[m] = make_float2(v.x * w, v.y * w);
            }
        }
        if (b == 0 && !(kMtdDma<P, BEAMS, LA, W>() && a.mti_lag <= 0)) after_loads();
        RSP_STAMP(1, 1, true);
        if constexpr (P >= kMtdLoadPrioMinP) __builtin_amdgcn_s_setprio(0);   // the tile's loads are out
        fft_reg_w<P, G, 1, E, 0, NW>(u, reinterpret_cast<float2*>(smem) + c * C::SLOT, g, tw);
        RSP_STAMP(1, 2, false);
        if constexpr (BEAMS == 2) {
            if (b == 0) {
#pragma unroll
                for (int m = 0; m < E; ++m) m0[m] = __builtin_amdgcn_sqrtf(fmaf(u[m].x, u[m].x, u[m].y * u[m].y));
            }
        }
    }

    // The flag plane's zero background for this tile (range stage on: the 1s come later from
    // the hit list): W columns x P rows, one 16-byte store per row segment, issued while the
    // FFT runs -- instead of a byte store per cell in the Doppler epilogue.
    bool bg_done = false;
    if constexpr (W % 16 == 0) {
        if (T.flag && a.cv.enabled && a.rflag && a.flag_zero && (R % 16u) == 0u) {
            typedef int v4i __attribute__((ext_vector_type(4)));
            const auto fz = buf_rsrc(T.flag, plane);
            constexpr int SEG = W / 16;
            for (int i = tx; i < P * SEG; i += C::T) {
                const int c0 = T.bx * W + (i % SEG) * 16;
                if (c0 < (int)R)
                    __builtin_amdgcn_raw_buffer_store_b128(v4i{0, 0, 0, 0}, fz, (uint32_t)(i / SEG) * R + (uint32_t)c0,
                                                           0u, SA);
            }
            bg_done = true;
        }
    }

    const auto dst = buf_rsrc(T.rdm, plane * 4u);
    const bool want_diff = BEAMS == 2 && T.diff != nullptr;
    const auto dfr = buf_rsrc(want_diff ? T.diff : nullptr, want_diff ? plane * 4u : 0u);
    const uint32_t vo_out = rv ? cell * 4u : kOob;
    const int srot = a.shift / G;
    float mg[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        int mm = m + srot;                // fftshift: bin g + G*m -> row g + G*mm
        if (mm >= E) mm -= E;
        float x = __builtin_amdgcn_sqrtf(fmaf(u[m].x, u[m].x, u[m].y * u[m].y));
        if constexpr (BEAMS == 2) {
            if (want_diff) buf_st_f(x - m0[m], dfr, vo_out, (uint32_t)(G * mm) * R * 4u);   // |R| - |L|
            x += m0[m];                                                                      // |L| + |R|
        }
        mg[m] = x;
        if constexpr (SA != 0) buf_st_fa<SA>(x, dst, vo_out, (uint32_t)(G * mm) * R * 4u);
        else buf_st_f_stream(x, dst, vo_out, (uint32_t)(G * mm) * R * 4u);
    }
    // fun_0v_pressing's zeroed rows [z_lo, z_hi) (the DMX zeroSetFlagMTD band wraps through row
    // 0: rows [0, z_hi - P) too), as a second store of 0 to the few of the thread's rows inside
    // the band -- the same thread's later store to the same address wins -- instead of a
    // compare-select on every row (one or two rows per thread; 4 VALU per row saved)
    const int zw = a.z_hi > P ? a.z_hi - P : 0;
    auto zero_rdm = [&](int mm) {   // (mm is per lane: the row offset goes in the VGPR offset)
        const uint32_t vz = rv ? (cell + (uint32_t)(G * mm) * R) * 4u : kOob;
        if constexpr (SA != 0) buf_st_fa<SA>(0.f, dst, vz, 0u);
        else buf_st_f_stream(0.f, dst, vz, 0u);
    };
    own_rows<G, E>(g, a.z_lo, a.z_hi, zero_rdm);
    own_rows<G, E>(g, 0, zw, zero_rdm);
    RSP_STAMP(1, 3, false);
    if (!a.cv.enabled) return;
    lds_barrier();  // the FFT exchange slots are free from here on
    float* mag = REF > 0 ? reinterpret_cast<float*>(smem) + c * C::MS2 + C::SPAD
                         : reinterpret_cast<float*>(smem) + c * C::MS;
#pragma unroll
    for (int m = 0; m < E; ++m) {
        int mm = m + srot;
        if (mm >= E) mm -= E;
        mag[g + G * mm] = mg[m];
    }
    // the CFAR input's zero rows (main_cfar.m:90-91) and the RDM's band, by the same second
    // write of 0 (LDS writes of one thread land in order)
    auto zero_mag = [&](int mm) { mag[g + G * mm] = 0.f; };
    own_rows<G, E>(g, a.z_lo, a.z_hi, zero_mag);
    own_rows<G, E>(g, 0, zw, zero_mag);
    own_rows<G, E>(g, a.cv.cz_lo, a.cv.cz_hi, zero_mag);
    lds_barrier();

    const int v0 = cfar_run<G, W>(g) * E;   // this thread's run of Doppler rows
    const bool col_on = rv && in_segs(r, a.cv.nseg, a.cv.seg_lo, a.cv.seg_hi);
    DopplerOut o;
    o.want_fv = T.flagV != nullptr;
    o.fused = T.flag != nullptr;
    o.coherent = SA != 0;
    o.rflag = a.rflag != 0;
    o.zero_bg = a.flag_zero != 0 && !bg_done;
    o.fv = buf_rsrc(o.want_fv ? T.flagV : nullptr, o.want_fv ? plane : 0u);
    o.fl = buf_rsrc(o.fused ? T.flag : nullptr, o.fused ? plane : 0u);
    o.vo = rv ? (uint32_t)v0 * R + (uint32_t)r : kOob;
    o.R = R;
    o.hits = T.hits;
    o.lds_count = s_hits;
    o.cell0 = T.cell_base + (uint32_t)v0 * R + (uint32_t)r;
    if constexpr (REF > 0) {
        doppler_cfar_fixed<P, REF, BEAMS>(mag, a.cv, col_on, v0, o);
    } else {
        float* sums = reinterpret_cast<float*>(smem) + W * C::MS + c * C::SMS + C::SPAD;
        doppler_sums(mag, sums, P, a.cv.ref, v0, v0 + E);
        lds_barrier();
        doppler_flags<E>(mag, sums, a.cv, col_on, v0, v0 + E, o);
    }
    RSP_STAMP(1, 4, false);
    if (o.fused && o.rflag) {
        lds_barrier();
        if (tx == 0) {
            if (SA != 0) st_u32_sc1(T.hit_count, *s_hits);
            else *T.hit_count = *s_hits;
        }
    }
}

// MTD: one workgroup = W range bins x all P pulses.  Thread (c, g): range bin c of the
// tile, pulses g + G*m (m < E) -- the strided pattern of fft_reg, so the pulse-compressed
// samples load straight into registers with W-wide coalesced rows, the slow-time FFT runs
// register-resident with LDS exchanges, and |X| leaves in coalesced RDM rows.  The fftshift
// offset is 0 or P/2, a multiple of G, so bin g + G*m lands in row g + G*((m + shift/G) mod E):
// a wave-uniform rotation, and every row offset is an SGPR operand of the buffer access.
// REF > 0: Doppler CFAR specialised on the reference window; REF == 0: runtime window.
// P is the Doppler FFT length; a CPI supplies a.pin <= P pulses per beam (rows past pin are
// the zero padding of fft(x, P, 1): out of the buffer's range, they load as 0).  BEAMS == 2:
// the DMX pair -- both beams' slow-time FFTs, RDM = |X_0| + |X_1|, diff = |X_1| - |X_0|.
// One MTD workgroup: tile bx (of gx along range) of launch CPI by (of gy); smem / s_hits: the
// workgroup's dynamic LDS and hit counter.
template <int P, int REF, int BEAMS, bool JOB>
__device__ __forceinline__ void mtd_block(const float2* __restrict__ pc, float* __restrict__ rdm,
                                          uint8_t* __restrict__ flagV, const MtdArgs& a, int bx, int by, int gx, int gy,
                                          unsigned char* smem, uint32_t* s_hits) {
    using C = MtdCfg<P, BEAMS>;
    const size_t cpi = (size_t)by;
    const size_t R = (size_t)a.R_out;
    const size_t plane = (size_t)P * R;
    size_t row0 = cpi * (size_t)a.pin * BEAMS;                   // first PC row of this CPI
    if (a.nwin > 0) row0 = (cpi / a.nwin) * (size_t)a.pin + a.win_start[cpi % a.nwin];
    const uint32_t wg = (uint32_t)by * (uint32_t)gx + (uint32_t)bx;
    MtdTile T;
    T.pc = pc + row0 * R;
    T.rdm = rdm + cpi * plane;
    T.diff = (BEAMS == 2 && a.diff) ? a.diff + cpi * plane : nullptr;
    T.flagV = flagV ? flagV + cpi * plane : nullptr;
    T.flag = a.flag ? a.flag + cpi * plane : nullptr;
    T.hits = a.hits ? a.hits + (size_t)wg * (C::W * P) : nullptr;
    T.hit_count = a.hit_count ? a.hit_count + wg : nullptr;
    T.cell_base = (uint32_t)(cpi * plane) + a.cell_off;
    T.bx = bx;
    if constexpr (C::W < 32) {   // 8 consecutive tiles on one XCD (workgroup x goes to XCD x % 8):
        // their partial RDM / flag row segments (W = 16: 64-B RDM and 16-B flag segments) meet
        // in one L2 and leave it as whole lines -- 8 tiles make the flag segments whole 128-B
        // lines too (c4 MTD 419 -> 397 us per launch, c4 +4.7 %; c5 neutral; 4 tiles: c5 +1.5-2 %
        // over none); 4 tiles when the row's tile count is not a multiple of 64.  (At W = 32 the
        // RDM segments are whole lines and grouping cost c3's MTD 3 %.)
        const int x = bx;
        if (gx % 64 == 0) T.bx = (x / 64) * 64 + (x % 8) * 8 + (x / 8) % 8;
        else if (gx % 32 == 0) T.bx = (x / 32) * 32 + (x % 8) * 4 + (x / 8) % 4;
    }
    const int nwg = gx * gy;
    // one instance of the tile (the kernel's code stays ~half the size: it shares the
    // instruction cache with the PC kernel of the other pipeline); the range job is runtime-
    // guarded -- with n == 0 its hook and finish() return at once
    const bool job = JOB && a.prev_nregions > 0 && a.prev_cr.ref == 5 && a.prev_cr.save == 7 && (int)wg < a.prev_nregions &&
                     (uint64_t)a.prev_nregions * (uint64_t)a.prev_region < (uint64_t)(kOob / 4u);
    RangeJob57 rj;
    const RangeSrc rs = RangeSrc::of(a);
    RSP_STAMP(1, 0, false);
    if constexpr (P >= kMtdLoadPrioMinP) __builtin_amdgcn_s_setprio(kMtdLoadPrio);
    RSP_STAMP_RT(1, 8);
    if (job) rj.fetch_idx(rs, (int)wg);
    if constexpr (JOB) mtd_tile<P, REF, BEAMS, 0, 0>(T, a, smem, s_hits, RangeHookT<0>{rj, rs});
    else mtd_tile<P, REF, BEAMS, 0, 0>(T, a, smem, s_hits, NoHook{});
    RSP_STAMP(1, 5, false);
    rj.finish(rs);
    RSP_STAMP(1, 6, false);
    if (job ? (rj.n > blockDim.x || a.prev_nregions > nwg) : a.prev_nregions > 0)
        prev_chunk_hits(a, (int)wg, nwg, job ? (int)blockDim.x : 0);
    RSP_STAMP(1, 7, true);
    RSP_STAMP_RT(1, 9);
}

// JOB: this launch carries the previous chunk's range stage for the reference's window (the
// RangeJob57 gathers ride on the tile load); otherwise prev_chunk_hits (if any) runs after the tile.
template <int P, int REF, int BEAMS, bool JOB>
__global__ __launch_bounds__((MtdCfg<P, BEAMS>::T), (MtdCfg<P, BEAMS>::WPE)) void mtd_kernel(const float2* __restrict__ pc,
                                                     float* __restrict__ rdm,
                                                     uint8_t* __restrict__ flagV, MtdArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ uint32_t s_hits;
    mtd_block<P, REF, BEAMS, JOB>(pc, rdm, flagV, a, (int)blockIdx.x, (int)blockIdx.y, (int)gridDim.x, (int)gridDim.y,
                                  smem, &s_hits);
}

// Slow-time DFT for a pulse count without a radix plan (the v2 native P = 332 = 4*83,
// MTD/main_produce_dataset_win_xzr_v2.m:31) by Bluestein's identity:
//   X[k] = c[k] sum_n (x[n] w[n] c[n]) conj(c[k-n]),   c[n] = exp(-j pi n^2 / P),
// a circular convolution of length NF >= 2P - 1 (power of two): FFT, multiply by the chirp's
// spectrum, FFT again (the inverse as conj(FFT(conj))).  |c[k]| = 1, so the magnitude
// needs no final chirp.  Bins k < P are kept; fftshift / 0-v / Doppler CFAR as mtd_kernel
// (runtime CFAR window), with per-element row offsets (P is not a multiple of G).
template <int NF>
__global__ __launch_bounds__(MtdCfg<NF>::T) void mtd_bluestein_kernel(const float2* __restrict__ pc,
                                                               float* __restrict__ rdm,
                                                               uint8_t* __restrict__ flagV, MtdArgs a) {
    using C = MtdCfg<NF>;
    constexpr int G = C::G, E = C::E, W = C::W;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ uint32_t s_hits;
    if (threadIdx.x == 0) s_hits = 0u;
    const int c = threadIdx.x % W, g = threadIdx.x / W;
    const size_t cpi = blockIdx.y;
    const uint32_t R = (uint32_t)a.R_out;
    const int r = blockIdx.x * W + c;
    const bool rv = r < (int)R;
    const int P = a.pin;
    const uint32_t plane = (uint32_t)P * R;
    size_t row0 = cpi * (size_t)P;
    if (a.nwin > 0) row0 = (cpi / a.nwin) * (size_t)P + a.win_start[cpi % a.nwin];
    const auto src = buf_rsrc(pc + row0 * R, plane * 8u);           // rows >= P load as 0
    const uint32_t vo_in = rv ? ((uint32_t)g * R + (uint32_t)r) * 8u : kOob;
    float2 u[E];
    if (a.mti_lag > 0) {   // fused MTI, as mtd_tile
        const int lag = a.mti_lag;
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const float2 v0 = buf_ld_f2(src, vo_in, (uint32_t)(G * m) * R * 8u);
            const float2 v1 = buf_ld_f2(src, vo_in, (uint32_t)(G * m + lag) * R * 8u);
            const float2 d = g + G * m + lag < P ? make_float2(v1.x - v0.x, v1.y - v0.y) : make_float2(0.f, 0.f);
            u[m] = cmul(d, a.bwc[g + G * m]);
        }
    } else {
#pragma unroll
        for (int m = 0; m < E; ++m)
            u[m] = cmul(buf_ld_f2(src, vo_in, (uint32_t)(G * m) * R * 8u), a.bwc[g + G * m]);
    }
    float2* slot = reinterpret_cast<float2*>(smem) + c * C::SLOT;
    fft_reg<NF, G, 1, E>(u, slot, g, a.tw);
#pragma unroll
    for (int m = 0; m < E; ++m) u[m] = cmul_conj(u[m], a.bspec[g + G * m]);   // conj(A .* B), 1/NF in B
    fft_reg<NF, G, 1, E>(u, slot, g, a.tw);                                  // conj of the convolution

    const auto dst = buf_rsrc(rdm + cpi * plane, plane * 4u);
    float mg[E];
    int vr[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const int k = g + G * m;                   // Doppler bin
        int v = k + a.shift;                       // fftshift: out[v] = X[(v - shift) mod P]
        if (v >= P) v -= P;
        float x = __builtin_amdgcn_sqrtf(fmaf(u[m].x, u[m].x, u[m].y * u[m].y));
        if (v >= a.z_lo && v < a.z_hi) x = 0.f;   // fun_0v_pressing
        mg[m] = x;
        vr[m] = k < P ? v : -1;
        if (k < P) buf_st_f(x, dst, rv ? ((uint32_t)v * R + (uint32_t)r) * 4u : kOob, 0u);
    }
    if (!a.cv.enabled) return;   // (no CFAR: no range stage pending either)
    __syncthreads();  // the FFT exchange slots are free from here on
    float* mag = reinterpret_cast<float*>(smem) + c * C::MS;
#pragma unroll
    for (int m = 0; m < E; ++m)
        if (vr[m] >= 0) mag[vr[m]] = (vr[m] >= a.cv.cz_lo && vr[m] < a.cv.cz_hi) ? 0.f : mg[m];
    __syncthreads();
    const int v0 = g * E, v1 = v0 + E < P ? v0 + E : P;    // this thread's run of Doppler rows
    const bool col_on = rv && in_segs(r, a.cv.nseg, a.cv.seg_lo, a.cv.seg_hi);
    DopplerOut o;
    o.want_fv = flagV != nullptr;
    o.fused = a.flag != nullptr;
    o.coherent = false;
    o.rflag = a.rflag != 0;
    o.zero_bg = a.flag_zero != 0;
    o.fv = buf_rsrc(o.want_fv ? flagV + cpi * plane : nullptr, o.want_fv ? plane : 0u);
    o.fl = buf_rsrc(o.fused ? a.flag + cpi * plane : nullptr, o.fused ? plane : 0u);
    o.vo = (rv && v0 < P) ? (uint32_t)v0 * R + (uint32_t)r : kOob;
    o.R = R;
    const uint32_t wg = blockIdx.y * gridDim.x + blockIdx.x;
    o.hits = a.hits ? a.hits + (size_t)wg * ((size_t)W * P) : nullptr;
    o.lds_count = &s_hits;
    o.cell0 = (uint32_t)cpi * plane + a.cell_off + (uint32_t)v0 * R + (uint32_t)r;
    float* sums = reinterpret_cast<float*>(smem) + W * C::MS + c * C::SMS + C::SPAD;
    doppler_sums(mag, sums, P, a.cv.ref, v0, v1);
    __syncthreads();
    doppler_flags<E>(mag, sums, a.cv, col_on, v0, v1, o);
    if (o.fused && o.rflag) {
        __syncthreads();
        if (threadIdx.x == 0) a.hit_count[wg] = s_hits;
    }
    if (a.prev_nregions > 0) prev_chunk_hits(a, (int)wg, (int)(gridDim.x * gridDim.y), 0);
}

template <int NF>
static hipError_t launch_mtd_bluestein(const float2* pc, float* rdm, uint8_t* flagV, int ncpi, const MtdArgs& a,
                                       hipStream_t s) {
    using C = MtdCfg<NF>;
    if (a.pin < 2 || 2 * a.pin - 1 > NF || a.beams != 1 || a.shift < 0 || a.shift >= a.pin) return hipErrorInvalidValue;
    if (a.cv.enabled && a.cv.save + a.cv.ref + 2 > C::SPAD) return hipErrorInvalidValue;
    if ((uint64_t)a.pin * a.R_out * 8 >= (uint64_t)kOob) return hipErrorInvalidValue;
    static LaunchOnce once;
    hipError_t e = lds_attr(once, (const void*)mtd_bluestein_kernel<NF>, C::lds);
    if (e != hipSuccess) return e;
    dim3 grid((unsigned)((a.R_out + C::W - 1) / C::W), (unsigned)ncpi),
        block(C::T);
    hipLaunchKernelGGL((mtd_bluestein_kernel<NF>), grid, block, C::lds, s, pc, rdm, flagV, a);
    return hipGetLastError();
}

int mtd_bluestein_nf(int P) {
    int nf = 64;
    while (nf < 2 * P - 1) nf <<= 1;
    return nf <= 2048 ? nf : 0;
}

template <int P, int REF, int BEAMS>
static hipError_t launch_mtd_pr(const float2* pc, float* rdm, uint8_t* flagV, int ncpi,
                                const MtdArgs& a, hipStream_t s) {
    using C = MtdCfg<P, BEAMS>;
    constexpr size_t lds = C::template lds_for<REF>();
    static LaunchOnce once, once_job;
    dim3 grid((unsigned)((a.R_out + C::W - 1) / C::W), (unsigned)ncpi),
        block(C::T);
    // the in-launch range job (RangeJob57) only for the reference's range window; any other
    // previous-chunk range stage runs as prev_chunk_hits in the no-job instance
    const bool job = REF > 0 && a.prev_nregions > 0 && a.prev_cr.ref == 5 && a.prev_cr.save == 7 &&
                     (uint64_t)a.prev_nregions * (uint64_t)a.prev_region < (uint64_t)(kOob / 4u);
    if constexpr (REF > 0) {
        if (job) {
            hipError_t e = lds_attr(once_job, (const void*)mtd_kernel<P, REF, BEAMS, true>, lds);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL((mtd_kernel<P, REF, BEAMS, true>), grid, block, lds, s, pc, rdm, flagV, a);
            return hipGetLastError();
        }
    }
    hipError_t e = lds_attr(once, (const void*)mtd_kernel<P, REF, BEAMS, false>, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((mtd_kernel<P, REF, BEAMS, false>), grid, block, lds, s, pc, rdm, flagV, a);
    return hipGetLastError();
}

template <int P, int BEAMS = 1>
static hipError_t launch_mtd_p(const float2* pc, float* rdm, uint8_t* flagV, int ncpi,
                               const MtdArgs& a, hipStream_t s) {
    using C = MtdCfg<P, BEAMS>;
    // shift is 0 or floor(P/2) = G*E/2; the row rotation needs it to be a multiple of G,
    // and the padded sums column needs save + ref + 2 <= SPAD
    if (a.shift % C::G != 0 || a.shift < 0 || a.shift >= P) return hipErrorInvalidValue;
    if (a.cv.enabled && a.cv.save + a.cv.ref + 2 > C::SPAD) return hipErrorInvalidValue;
    if ((uint64_t)P * a.R_out * 8 >= (uint64_t)kOob) return hipErrorInvalidValue;
    if (a.pin < 1 || a.pin > P || a.beams != BEAMS) return hipErrorInvalidValue;
    if (a.cv.enabled && a.cv.ref == 5 && a.cv.save == 7) return launch_mtd_pr<P, 5, BEAMS>(pc, rdm, flagV, ncpi, a, s);
    return launch_mtd_pr<P, 0, BEAMS>(pc, rdm, flagV, ncpi, a, s);
}

// Hit-list regions of one MTD launch: one per workgroup (tile of W range bins), W * rows
// entries each -- the tile's own cells, so a region can never overflow.
template <int P, int BEAMS>
static void mtd_regions_p(int rows, int R_out, int ncpi, int* nregions, int* region) {
    using C = MtdCfg<P, BEAMS>;
    *nregions = ((R_out + C::W - 1) / C::W) * ncpi;
    *region = C::W * rows;
}

void mtd_regions(int P, int R_out, int ncpi, int* nregions, int* region, int beams) {
    *nregions = 0;
    *region = 0;
    if (beams == 1 && !mtd_size_supported(P, 1)) {   // Bluestein: NF-point tiles, P rows kept
        switch (mtd_bluestein_nf(P)) {
#define RSP_MB(nf) case nf: mtd_regions_p<nf, 1>(P, R_out, ncpi, nregions, region); break;
            RSP_MB(64) RSP_MB(128) RSP_MB(256) RSP_MB(512) RSP_MB(1024) RSP_MB(2048)
#undef RSP_MB
            default: break;
        }
        return;
    }
    if (beams == 2) {
        switch (P) {
            case 512: mtd_regions_p<512, 2>(P, R_out, ncpi, nregions, region); break;
            case 1024: mtd_regions_p<1024, 2>(P, R_out, ncpi, nregions, region); break;
            case 2048: mtd_regions_p<2048, 2>(P, R_out, ncpi, nregions, region); break;
            default: break;
        }
        return;
    }
    switch (P) {
#define RSP_MR(p) case p: mtd_regions_p<p, 1>(P, R_out, ncpi, nregions, region); break;
        RSP_MR(16) RSP_MR(32) RSP_MR(64) RSP_MR(128) RSP_MR(256) RSP_MR(512) RSP_MR(1024)
        RSP_MR(2048) RSP_MR(48) RSP_MR(96) RSP_MR(192) RSP_MR(384) RSP_MR(768) RSP_MR(1536)
#undef RSP_MR
        default: break;
    }
}

bool mtd_size_supported(int P, int beams) {
    if (beams == 2) return P == 512 || P == 1024 || P == 2048;   // the DMX pair (mtd_FFT_num 2048)
    if (beams != 1) return false;
    switch (P) {
        case 16: case 32: case 64: case 128: case 256: case 512: case 1024: case 2048:
        case 48: case 96: case 192: case 384: case 768: case 1536:
            return true;
        default:
            return false;
    }
}

hipError_t launch_mtd(const float2* pc, float* rdm, uint8_t* flagV, int ncpi, const MtdArgs& a,
                      hipStream_t s) {
    if (ncpi <= 0) return hipSuccess;
    if (a.bnf > 0) {
        switch (a.bnf) {
            case 64: return launch_mtd_bluestein<64>(pc, rdm, flagV, ncpi, a, s);
            case 128: return launch_mtd_bluestein<128>(pc, rdm, flagV, ncpi, a, s);
            case 256: return launch_mtd_bluestein<256>(pc, rdm, flagV, ncpi, a, s);
            case 512: return launch_mtd_bluestein<512>(pc, rdm, flagV, ncpi, a, s);
            case 1024: return launch_mtd_bluestein<1024>(pc, rdm, flagV, ncpi, a, s);
            case 2048: return launch_mtd_bluestein<2048>(pc, rdm, flagV, ncpi, a, s);
            default: return hipErrorInvalidValue;
        }
    }
    if (a.beams == 2) {
        switch (a.P) {
            case 512: return launch_mtd_p<512, 2>(pc, rdm, flagV, ncpi, a, s);
            case 1024: return launch_mtd_p<1024, 2>(pc, rdm, flagV, ncpi, a, s);
            case 2048: return launch_mtd_p<2048, 2>(pc, rdm, flagV, ncpi, a, s);
            default: return hipErrorInvalidValue;
        }
    }
    switch (a.P) {
        case 16: return launch_mtd_p<16>(pc, rdm, flagV, ncpi, a, s);
        case 32: return launch_mtd_p<32>(pc, rdm, flagV, ncpi, a, s);
        case 64: return launch_mtd_p<64>(pc, rdm, flagV, ncpi, a, s);
        case 128: return launch_mtd_p<128>(pc, rdm, flagV, ncpi, a, s);
        case 256: return launch_mtd_p<256>(pc, rdm, flagV, ncpi, a, s);
        case 512: return launch_mtd_p<512>(pc, rdm, flagV, ncpi, a, s);
        case 1024: return launch_mtd_p<1024>(pc, rdm, flagV, ncpi, a, s);
        case 2048: return launch_mtd_p<2048>(pc, rdm, flagV, ncpi, a, s);
        case 48: return launch_mtd_p<48>(pc, rdm, flagV, ncpi, a, s);
        case 96: return launch_mtd_p<96>(pc, rdm, flagV, ncpi, a, s);
        case 192: return launch_mtd_p<192>(pc, rdm, flagV, ncpi, a, s);
        case 384: return launch_mtd_p<384>(pc, rdm, flagV, ncpi, a, s);
        case 768: return launch_mtd_p<768>(pc, rdm, flagV, ncpi, a, s);
        case 1536: return launch_mtd_p<1536>(pc, rdm, flagV, ncpi, a, s);
        default: return hipErrorInvalidValue;
    }
}

// (Round 5's persistent one-launch PC -> MTD dataflow, flow_kernel / rsp_set_flow, measured 82 %
// of the chunked chain at c3 and left the product in round 6: DESIGN.md §7c / §7d; its source is
// in the history, commit e3a7a73.  Round 6's split form -- a PC-only and an MTD-only persistent
// kernel on CU-masked streams -- measured 75.6 % (profiles/r06/flow2/ab_record.txt, commit
// d7d9bbe).  The sc1 (LA / SA) and opaque-index (OPQ) variants of the tile and range-job templates
// above are what they instantiated.)

// ================================================================== Doppler CFAR from an RDM
// rsp_cfar's first stage: tile of W columns x V rows staged column-major in LDS.
__global__ __launch_bounds__(kBlock) void cfar_v_kernel(const float* __restrict__ rdm,
                                                        uint8_t* __restrict__ flagV, int V, int R,
                                                        int lw, CfarVArgs cv) {
    extern __shared__ __attribute__((aligned(16))) float magv[];
    const int W = 1 << lw, G = kBlock >> lw;
    const int c = threadIdx.x & (W - 1), g = threadIdx.x >> lw;
    const size_t cpi = blockIdx.y;
    const int r = blockIdx.x * W + c;
    const bool rv = r < R;
    const int ms = V + 1;
    float* mag = magv + c * ms;
    float* sums = magv + W * ms + c * ms;
    const float* src = rdm + cpi * (size_t)V * R + (rv ? r : 0);
    for (int v = g; v < V; v += G)
        mag[v] = (rv && !(v >= cv.cz_lo && v < cv.cz_hi)) ? src[(size_t)v * R] : 0.f;
    __syncthreads();
    const int run = (V + G - 1) / G;
    const int v0 = g * run, v1 = v0 + run < V ? v0 + run : V;
    doppler_sums(mag, sums, V, cv.ref, v0, v1);
    __syncthreads();
    const bool col_on = rv && in_segs(r, cv.nseg, cv.seg_lo, cv.seg_hi);
    doppler_flags(mag, sums, cv, col_on, v0, v1, flagV + cpi * (size_t)V * R + r, R, rv);
}

hipError_t launch_cfar_v(const float* rdm, uint8_t* flagV, int ncpi, int V, int R,
                         const CfarVArgs& a, hipStream_t s) {
    if (ncpi <= 0) return hipSuccess;
    int lw = 6;
    while (lw > 0 && (size_t)2 * (1 << lw) * (V + 1) * sizeof(float) > 96 * 1024) --lw;
    const size_t lds = (size_t)2 * (1 << lw) * (V + 1) * sizeof(float);
    static LaunchOnce once;
    hipError_t e = lds_attr(once, (const void*)cfar_v_kernel, 160 * 1024);
    if (e != hipSuccess) return e;
    dim3 grid((unsigned)((R + (1 << lw) - 1) >> lw), (unsigned)ncpi), block(kBlock);
    hipLaunchKernelGGL(cfar_v_kernel, grid, block, lds, s, rdm, flagV, V, R, lw, a);
    return hipGetLastError();
}

// ================================================================== range CFAR + re-localisation
// One workgroup per RDM row.  Phase 1 stages the row (+ zero halo) and its Doppler flags in
// LDS; phase 2 forms the range window sums; phase 3 evaluates the range CFAR at every cell
// (Function_CFAR1D_sub_fixCells.m:34-58 -- the decision at a cell does not depend on which
// hit asked for it); phase 4 resolves executeCFAR.m:45-84 as a gather: cell c is flagged iff
// some Doppler hit r in {c-1, c, c+1} of c's segment picks c as the first maximum among its
// passing cells {r-1, r, r+1}.  Each thread handles 4 adjacent cells per step, so flags
// leave as coalesced 32-bit words.
constexpr int kHalo = 32;   // >= guard + ref + 2 (checked on the host)

__global__ __launch_bounds__(kBlock) void cfar_r_generic_kernel(const float* __restrict__ rdm,
                                                        const uint8_t* __restrict__ flagV,
                                                        uint8_t* __restrict__ flag, CfarRArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int t = threadIdx.x;
    const int v = blockIdx.x;
    const size_t cpi = blockIdx.y;
    const int R = a.R;
    const size_t rowoff = (cpi * (size_t)a.V + v) * (size_t)R;
    uint8_t* out = flag + rowoff;
    if (v < a.lo || v >= a.hi) {
        for (int c = t; c < R; c += kBlock) out[c] = 0;
        return;
    }
    const uint8_t* fv_g = flagV + rowoff;
    if (!a.rflag) {
        for (int c = t; c < R; c += kBlock) out[c] = fv_g[c];
        return;
    }
    const int Rp = (R + 3) & ~3;                      // row length rounded to words
    const int L = Rp + 2 * kHalo;
    float* xs = reinterpret_cast<float*>(smem) + kHalo;          // xs[-kHalo, Rp + kHalo)
    float* ss = xs + L;                                            // window sums, same indexing
    uint8_t* pass = reinterpret_cast<uint8_t*>(ss - kHalo + L) + kHalo;   // pass[-kHalo, Rp+kHalo)
    uint8_t* fv = pass + L;                                        // fv[-kHalo, Rp+kHalo)
    const bool zrow = (v >= a.cz_lo && v < a.cz_hi);
    const float* xr = rdm + rowoff;
    for (int i = t; i < L; i += kBlock) {
        const int c = i - kHalo;
        const bool in = c >= 0 && c < R;
        xs[c] = (in && !zrow) ? xr[c] : 0.f;
        fv[c] = in ? fv_g[c] : 0;
        pass[c] = 0;
    }
    __syncthreads();
    const int ref = a.ref;
    for (int i = t; i < L; i += kBlock) {
        const int c = i - kHalo;
        if (c + ref > Rp + kHalo) continue;
        float s = 0.f;
        for (int k = 0; k < ref; ++k) s += xs[c + k];
        ss[c] = s;
    }
    __syncthreads();
    for (int c = t; c < R; c += kBlock) {
        int slo, shi;
        seg_of(c, a.nseg, a.seg_lo, a.seg_hi, slo, shi);
        uint8_t p = 0;
        if (shi > slo) {
            const int l1 = c - a.save - ref, r1 = c + a.save + 1;
            const bool lok = l1 >= slo, rok = r1 + ref <= shi;
            p = cfar_test(xs[c], lok ? ss[l1] : 0.f, rok ? ss[r1] : 0.f, lok, rok, a.method, a.Tr);
        }
        pass[c] = p;
    }
    __syncthreads();
    for (int c0 = 4 * t; c0 < R; c0 += 4 * kBlock) {
        // x, pass at c0-2 .. c0+5 and fv at c0-1 .. c0+4, from aligned words
        float xw[12];
        const float4 xa = *reinterpret_cast<const float4*>(xs + c0 - 4);
        const float4 xb = *reinterpret_cast<const float4*>(xs + c0);
        const float4 xc = *reinterpret_cast<const float4*>(xs + c0 + 4);
        xw[0] = xa.x; xw[1] = xa.y; xw[2] = xa.z; xw[3] = xa.w;
        xw[4] = xb.x; xw[5] = xb.y; xw[6] = xb.z; xw[7] = xb.w;
        xw[8] = xc.x; xw[9] = xc.y; xw[10] = xc.z; xw[11] = xc.w;
        const uint32_t pa = *reinterpret_cast<const uint32_t*>(pass + c0 - 4);
        const uint32_t pb = *reinterpret_cast<const uint32_t*>(pass + c0);
        const uint32_t pcw = *reinterpret_cast<const uint32_t*>(pass + c0 + 4);
        const uint32_t fa = *reinterpret_cast<const uint32_t*>(fv + c0 - 4);
        const uint32_t fb = *reinterpret_cast<const uint32_t*>(fv + c0);
        const uint32_t fc = *reinterpret_cast<const uint32_t*>(fv + c0 + 4);
        const uint64_t pw = (uint64_t)pa | ((uint64_t)pb << 32);   // byte k <-> cell c0-4+k
        const uint64_t fw = (uint64_t)fa | ((uint64_t)fb << 32);
        auto P_ = [&](int k) -> bool {   // pass at cell c0-4+k, k in [0, 12)
            return k < 8 ? ((pw >> (8 * k)) & 0xff) != 0 : ((pcw >> (8 * (k - 8))) & 0xff) != 0;
        };
        auto F_ = [&](int k) -> bool {
            return k < 8 ? ((fw >> (8 * k)) & 0xff) != 0 : ((fc >> (8 * (k - 8))) & 0xff) != 0;
        };
        uint32_t word = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = c0 + j;
            int slo, shi;
            seg_of(c, a.nseg, a.seg_lo, a.seg_hi, slo, shi);
            bool f = false;
#pragma unroll
            for (int d = -1; d <= 1; ++d) {
                const int rr = c + d;   // a Doppler hit at rr tests cells rr-1 .. rr+1
                if (rr < slo || rr >= shi || !F_(4 + j + d)) continue;
                int best = -100;
                float bx = 0.f;
#pragma unroll
                for (int e = -1; e <= 1; ++e) {
                    const int q = rr + e;
                    const int k = 4 + j + d + e;
                    if (q < slo || q >= shi || !P_(k)) continue;
                    if (best == -100 || xw[k] > bx) { best = d + e; bx = xw[k]; }   // first max
                }
                f |= (best == 0);
            }
            if (c < R && f) word |= 1u << (8 * j);
        }
        if (c0 + 3 < R && (R & 3) == 0) {
            *reinterpret_cast<uint32_t*>(out + c0) = word;
        } else {
            for (int j = 0; j < 4 && c0 + j < R; ++j) out[c0 + j] = (word >> (8 * j)) & 0xff;
        }
    }
}


// Range CFAR specialised on the window (REF reference + SAVE guard cells; the reference
// uses 5 + 7): no LDS and no barriers.  Thread = 4 adjacent cells c0..c0+3 of one row; it
// reads x[c0-16, c0+20) as aligned float4s from L2 (neighbouring threads overlap in L1),
// forms the 16 window sums it needs in MATLAB's summation order, evaluates the range test
// at c0-2 .. c0+5 and resolves the four outputs as in cfar_r_generic_kernel.  Cells whose
// windows cross a segment edge take the segment-aware branch.
// Range CFAR + re-localisation for the 4 cells c0..c0+3 of one RDM row (slow path: some
// Doppler hit in c0-1..c0+4).  fa/fb/fc: flagV words of cells c0-4.., c0.., c0+4.. .
template <int REF, int SAVE>
__device__ __forceinline__ uint32_t cfar4(const float* __restrict__ xr, uint32_t fa, uint32_t fb, uint32_t fc,
                                          int c0, int R, bool zrow, const CfarRArgs& a) {
    constexpr int H = SAVE + REF + 2;          // farthest x offset a result depends on
    constexpr int B = (H + 3) & ~3;            // aligned halo
    constexpr int NX = 4 + 2 * B;              // x values held per thread
    float x[NX];   // x[k] = row[c0 - B + k]
#pragma unroll
    for (int k = 0; k < NX; k += 4) {
        const int c = c0 - B + k;
        float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
        if (!zrow && c >= 0 && c + 3 < R) q = *reinterpret_cast<const float4*>(xr + c);
        x[k] = q.x; x[k + 1] = q.y; x[k + 2] = q.z; x[k + 3] = q.w;
    }
    int slo, shi;
    seg_of(c0, a.nseg, a.seg_lo, a.seg_hi, slo, shi);
    const bool simple = (c0 - H >= slo) && (c0 + 3 + H < shi);   // all windows inside one segment
    bool pass[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {   // cell q = c0 - 2 + i, x index B - 2 + i
        const int xi = B - 2 + i;
        float sl = 0.f, sr = 0.f;
#pragma unroll
        for (int k = 0; k < REF; ++k) sl += x[xi - SAVE - REF + k];
#pragma unroll
        for (int k = 0; k < REF; ++k) sr += x[xi + SAVE + 1 + k];
        if (simple) {
            pass[i] = x[xi] >= (a.method == 0 ? fmaxf(sl, sr) : fminf(sl, sr)) * a.Tr;
        } else {
            const int q = c0 - 2 + i;
            int ql, qh;
            seg_of(q, a.nseg, a.seg_lo, a.seg_hi, ql, qh);
            const bool lok = q - SAVE - REF >= ql, rok = q + SAVE + REF < qh;
            pass[i] = (qh > ql) && cfar_test(x[xi], sl, sr, lok, rok, a.method, a.Tr);
        }
    }
    const uint64_t fw = (uint64_t)fa | ((uint64_t)fb << 32);   // byte k <-> cell c0 - 4 + k
    uint32_t word = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = c0 + j;
        int cl = slo, ch = shi;
        if (!simple) seg_of(c, a.nseg, a.seg_lo, a.seg_hi, cl, ch);
        bool f = false;
#pragma unroll
        for (int d = -1; d <= 1; ++d) {
            const int rr = c + d;
            const int fk = 4 + j + d;
            const bool hit = fk < 8 ? ((fw >> (8 * fk)) & 0xff) != 0 : ((fc >> (8 * (fk - 8))) & 0xff) != 0;
            if (!hit || rr < cl || rr >= ch) continue;
            int best = -100;
            float bx = 0.f;
#pragma unroll
            for (int e = -1; e <= 1; ++e) {
                const int q = rr + e;
                const int i = 2 + j + d + e;   // pass/x index of cell q
                if (q < cl || q >= ch || !pass[i]) continue;
                const float xv = x[B - 2 + i];
                if (best == -100 || xv > bx) { best = d + e; bx = xv; }   // first max
            }
            f |= (best == 0);
        }
        if (f) word |= 1u << (8 * j);
    }
    return word;
}

template <int REF, int SAVE>
__global__ __launch_bounds__(kBlock) void cfar_r_kernel(const float* __restrict__ rdm,
                                                        const uint8_t* __restrict__ flagV,
                                                        uint8_t* __restrict__ flag, CfarRArgs a, int groups) {
    const int R = a.R;
    const int v = blockIdx.x / groups;
    const int c0 = ((blockIdx.x % groups) * kBlock + threadIdx.x) * 4;
    if (c0 >= R) return;
    const size_t cpi = blockIdx.y;
    const size_t rowoff = (cpi * (size_t)a.V + v) * (size_t)R;
    uint32_t* out = reinterpret_cast<uint32_t*>(flag + rowoff + c0);
    if (v < a.lo || v >= a.hi) {
        *out = 0u;
        return;
    }
    const uint32_t* fvw = reinterpret_cast<const uint32_t*>(flagV + rowoff);
    const uint32_t fa = c0 >= 4 ? fvw[c0 / 4 - 1] : 0u;
    const uint32_t fb = fvw[c0 / 4];
    const uint32_t fc = c0 + 4 < R ? fvw[c0 / 4 + 1] : 0u;
    if ((fa >> 24) == 0 && fb == 0 && (fc & 0xff) == 0) {   // no Doppler hit can reach these cells
        *out = 0u;
        return;
    }
    *out = cfar4<REF, SAVE>(rdm + rowoff, fa, fb, fc, c0, R, v >= a.cz_lo && v < a.cz_hi, a);
}

// 16 cells per thread (R % 16 == 0): one 16-B flagV load, the neighbouring groups' edge
// words from the adjacent lanes, one 16-B flag store; the 4-cell slow path runs only for
// groups with a Doppler hit within reach.  Hits are sparse, so this is the streaming pass
// over flagV -> flag at a quarter of the waves and memory instructions of cfar_r_kernel.
template <int REF, int SAVE>
__global__ __launch_bounds__(kBlock) void cfar_r16_kernel(const float* __restrict__ rdm,
                                                          const uint8_t* __restrict__ flagV,
                                                          uint8_t* __restrict__ flag, CfarRArgs a, int groups) {
    const int R = a.R;
    const int v = blockIdx.x / groups;
    const int c0 = ((blockIdx.x % groups) * kBlock + threadIdx.x) * 16;
    const bool in = c0 < R;
    const size_t cpi = blockIdx.y;
    const size_t rowoff = (cpi * (size_t)a.V + v) * (size_t)R;
    const bool row_on = v >= a.lo && v < a.hi;
    if (!in) return;
    // this group's 16 flags and the edge words of the neighbouring groups, all in one round
    // trip (the neighbours' words sit in the cache lines the adjacent lanes fetch anyway)
    uint4 f = make_uint4(0u, 0u, 0u, 0u);
    uint32_t left = 0u, right = 0u;
    if (row_on) {
        const uint8_t* fr = flagV + rowoff;
        f = *reinterpret_cast<const uint4*>(fr + c0);
        if (c0 >= 16) left = *reinterpret_cast<const uint32_t*>(fr + c0 - 4);
        if (c0 + 16 < R) right = *reinterpret_cast<const uint32_t*>(fr + c0 + 16);
    }
    uint4 o = make_uint4(0u, 0u, 0u, 0u);
    if (row_on && ((left >> 24) | f.x | f.y | f.z | f.w | (right & 0xff)) != 0) {
        const float* xr = rdm + rowoff;
        const bool zrow = v >= a.cz_lo && v < a.cz_hi;
        const uint32_t w[6] = {left, f.x, f.y, f.z, f.w, right};
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const uint32_t fa = w[g], fb = w[g + 1], fc = w[g + 2];
            uint32_t r = 0u;
            if ((fa >> 24) != 0 || fb != 0 || (fc & 0xff) != 0) r = cfar4<REF, SAVE>(xr, fa, fb, fc, c0 + 4 * g, R, zrow, a);
            (g == 0 ? o.x : g == 1 ? o.y : g == 2 ? o.z : o.w) = r;
        }
    }
    *reinterpret_cast<uint4*>(flag + rowoff + c0) = o;
}

// Scatter form of the range stage: one thread per Doppler hit (v, r) of the MTD kernel's
// list.  Candidates q in {r-1, r, r+1} within r's column segment take the range CFAR test
// (Function_CFAR1D_sub_fixCells.m:34-58, one-sided fallback at segment edges); the first
// maximum among passing candidates gets flag 1 (executeCFAR.m:64-84).  Several hits may
// pick one cell; the writes are all 1.  Window sums are direct left-to-right adds.
// One workgroup per region (a region is one MTD workgroup's hits: up to W*P entries, ~470
// per region at c5, whose 0-v band edges fire in every column), its threads striding the list.
constexpr int kHitThreads = 256;

template <int REF, int SAVE>
__global__ __launch_bounds__(kHitThreads) void cfar_hits_kernel(const float* __restrict__ rdm,
                                                                uint8_t* __restrict__ flag,
                                                                const uint32_t* __restrict__ hits,
                                                                const uint32_t* __restrict__ counts, int nregions,
                                                                int region, CfarRArgs a) {
    cfar_hit_region<REF, SAVE>(rdm, flag, hits, counts, (int)blockIdx.x, region, a, (int)threadIdx.x, kHitThreads);
}

// The reference's window (5 reference + 7 guard cells): LPR lanes per hit region (LPR = 64: one
// wave per region, four regions per workgroup).  A region is one MTD tile's hit list (~10-50 hits
// at c3-c5), so a workgroup per region left most of its threads idle and took one dependent
// round-trip chain (count -> index -> cells) per region; here the count and the lane's first index
// load together (the index is in bounds past the count: a region holds W*P >= 256 entries), the
// lane's 17 cells follow as one batch of range-checked buffer loads (RangeJob57's gathers), and
// hits past the first LPR of a region follow in further batches the same way (the batch loop runs
// while any region of the wave has hits left, so every lane of the wave issues the gathers).
template <int LPR>
__global__ __launch_bounds__(kHitThreads) void cfar_hits57_kernel(const float* __restrict__ rdm,
                                                                  uint8_t* __restrict__ flag,
                                                                  const uint32_t* __restrict__ hits,
                                                                  const uint32_t* __restrict__ counts, int nregions,
                                                                  int region, CfarRArgs a) {
    // LPR <= 64: 64 / LPR regions per wave; LPR > 64 (a multiple of 64): a region spans LPR / 64
    // waves (the dense lists of 8192-cell regions, c5)
    constexpr int RPW = LPR >= 64 ? 1 : 64 / LPR;
    const int lane = (int)(threadIdx.x % 64);
    const int rg = LPR > 64 ? (int)(blockIdx.x * (kHitThreads / LPR) + threadIdx.x / LPR)
                            : (int)((blockIdx.x * (kHitThreads / 64) + threadIdx.x / 64) * RPW) + lane / LPR;
    if constexpr (RPW == 1) {
        if (rg >= nregions) return;   // (wave-uniform; no barriers below)
    }
    const int k = LPR > 64 ? (int)(threadIdx.x % LPR) : lane % LPR;
    constexpr int NX = RangeJob57::NX;
    const bool live = rg < nregions;
    const uint32_t* list = hits + (size_t)(live ? rg : 0) * region;
    const uint32_t n = live ? counts[rg] : 0u;
    uint32_t idx = list[k];
    const uint32_t R = (uint32_t)a.R, V = (uint32_t)a.V;
    const auto rr = buf_rsrc(rdm, kOob);
    // batches of LPR hits per region, one per lane; the next batch's index is loaded before this
    // batch's cells, so its round trip overlaps the gathers
    for (uint32_t b0 = 0;; b0 += LPR) {
        if constexpr (RPW == 1) {
            if (b0 >= n) break;
        } else {
            if (__ballot(b0 < n) == 0) break;
        }
        const bool mine = b0 + (uint32_t)k < n;
        const uint32_t nk = b0 + (uint32_t)LPR + (uint32_t)k;
        const uint32_t next = nk < n ? list[nk] : 0u;
        const uint32_t row = idx / R;
        const int r = (int)(idx - row * R);
        const int v = (int)(row % V);
        const bool zrow = v >= a.cz_lo && v < a.cz_hi;
        float x[NX];
        RangeJob57::gather(x, rr, row, r, mine && !zrow, a.R);
        if (mine) {
            int slo, shi;
            seg_of(r, a.nseg, a.seg_lo, a.seg_hi, slo, shi);
            if (shi > slo) {
                const int best = RangeJob57::test(x, r, slo, shi, a);
                if (best >= 0) flag[(size_t)row * R + best] = 1;
            }
        }
        idx = next;
    }
}

// Regions larger than 4096 cells (P = 512 tiles: c5's ~460 hits per region) take a workgroup
// each with the batched, branch-free gathers of cfar_hits57_kernel: c5 range stage 64 -> 50 us per
// 16-CPI group, +0.9 % (profiles/r05/ab/range_stage_grouping.txt).  Dev A/B: RSP_HITS_BIG=0
// restores the per-hit loads of cfar_hits_kernel.
static bool hits_big() {
    static const bool b = [] { const char* v = getenv("RSP_HITS_BIG"); return !(v && *v == '0'); }();
    return b;
}

hipError_t launch_cfar_hits(const float* rdm, uint8_t* flag, const uint32_t* hits, const uint32_t* counts,
                            int nregions, int region, const CfarRArgs& a, hipStream_t s) {
    if (nregions <= 0) return hipSuccess;
    // (the chunk's RDM holds nregions * region cells: byte offsets stay below the range check).
    // Hits per region grow with the tile's pulse count: regions of up to 4096 cells (c3: ~10
    // hits, c4: ~50) take a wave each (c4: 44 -> 31 us per launch, c3 unchanged); the 8192-cell
    // regions of P = 512 (c5: ~460 hits) keep a workgroup each (a wave took 12 -> 22 us).
    if (a.ref == 5 && a.save == 7 && region >= 64 && region <= 4096 &&
        (uint64_t)nregions * (uint64_t)region < (uint64_t)(kOob / 4u)) {
        // lanes per region: 16 for the sparse hit lists of tiles of <= 128 Doppler rows (c3: ~11
        // hits per region, range stage 37.5 -> 29.2 us per 16-chunk group, c3 +1.3 %), a wave for
        // longer tiles (c4: ~50 hits, 46.6 us at 64 lanes against 50.1 at 32 and 56.0 at 16;
        // profiles/r05/ab/range_stage_grouping.txt).  Dev A/B: environment RSP_HITS_LPR.
        static const int lpr_env = [] { const char* v = getenv("RSP_HITS_LPR"); return v && *v ? atoi(v) : 0; }();
        const int lpr = lpr_env > 0 ? lpr_env : (a.V <= 128 ? 16 : 64);
        auto go = [&](auto kern, int rpw) {
            const int rpb = (kHitThreads / 64) * rpw;   // regions per workgroup
            hipLaunchKernelGGL(kern, dim3((unsigned)((nregions + rpb - 1) / rpb)), dim3(kHitThreads), 0, s, rdm, flag,
                               hits, counts, nregions, region, a);
        };
        if (lpr == 16) go(cfar_hits57_kernel<16>, 4);
        else if (lpr == 32) go(cfar_hits57_kernel<32>, 2);
        else go(cfar_hits57_kernel<64>, 1);
    } else if (a.ref == 5 && a.save == 7 && region >= kHitThreads && hits_big() &&
               (uint64_t)nregions * (uint64_t)region < (uint64_t)(kOob / 4u)) {
        // larger regions: the batched gathers with the whole workgroup on a region
        hipLaunchKernelGGL(cfar_hits57_kernel<kHitThreads>, dim3((unsigned)nregions), dim3(kHitThreads), 0, s, rdm, flag,
                           hits, counts, nregions, region, a);
    } else if (a.ref == 5 && a.save == 7)   // the reference's parameters
        hipLaunchKernelGGL((cfar_hits_kernel<5, 7>), dim3((unsigned)nregions), dim3(kHitThreads), 0, s, rdm, flag,
                           hits, counts, nregions, region, a);
    else
        hipLaunchKernelGGL((cfar_hits_kernel<0, 0>), dim3((unsigned)nregions), dim3(kHitThreads), 0, s, rdm, flag,
                           hits, counts, nregions, region, a);
    return hipGetLastError();
}

// The window-specialised range kernels need no LDS; cfar_r_generic_kernel stages a row (+ halo)
// as x, window sums, pass and flagV bytes: 10 bytes per cell (none when rflag == 0: it copies flagV).
static bool cfar_r_specialised(const CfarRArgs& a) { return a.ref == 5 && a.save == 7 && a.rflag && (a.R & 3) == 0; }
static size_t cfar_r_generic_lds(const CfarRArgs& a) {
    return a.rflag ? (size_t)(((a.R + 3) & ~3) + 2 * kHalo) * (2 * sizeof(float) + 2) : 0;
}
bool cfar_r_supported(const CfarRArgs& a) { return cfar_r_specialised(a) || cfar_r_generic_lds(a) <= 160 * 1024; }

hipError_t launch_cfar_r(const float* rdm, const uint8_t* flagV, uint8_t* flag, int ncpi,
                         const CfarRArgs& a, hipStream_t s) {
    if (ncpi <= 0) return hipSuccess;
    if (!cfar_r_supported(a)) return hipErrorInvalidValue;
    const size_t lds = cfar_r_generic_lds(a);
    static LaunchOnce once;
    hipError_t e = lds_attr(once, (const void*)cfar_r_generic_kernel, 160 * 1024);
    if (e != hipSuccess) return e;
    if (a.ref == 5 && a.save == 7 && a.rflag && (a.R & 15) == 0) {   // the reference's parameters
        const int groups = (a.R / 16 + kBlock - 1) / kBlock;
        dim3 grid((unsigned)(groups * a.V), (unsigned)ncpi), block(kBlock);
        hipLaunchKernelGGL((cfar_r16_kernel<5, 7>), grid, block, 0, s, rdm, flagV, flag, a, groups);
        return hipGetLastError();
    }
    if (a.ref == 5 && a.save == 7 && a.rflag && (a.R & 3) == 0) {
        const int groups = (a.R / 4 + kBlock - 1) / kBlock;
        dim3 grid((unsigned)(groups * a.V), (unsigned)ncpi), block(kBlock);
        hipLaunchKernelGGL((cfar_r_kernel<5, 7>), grid, block, 0, s, rdm, flagV, flag, a, groups);
        return hipGetLastError();
    }
    dim3 grid((unsigned)a.V, (unsigned)ncpi), block(kBlock);
    hipLaunchKernelGGL(cfar_r_generic_kernel, grid, block, lds, s, rdm, flagV, flag, a);
    return hipGetLastError();
}

// ================================================================== ingest / transposes
__device__ __forceinline__ float2 ld_el(const float2* p) { return *p; }
__device__ __forceinline__ float2 ld_el(const __half2* p) { return __half22float2(*p); }
__device__ __forceinline__ float2 ld_el(const double2* p) { return ld_c(p); }
__device__ __forceinline__ float ld_el(const float* p) { return *p; }
__device__ __forceinline__ uint8_t ld_el(const uint8_t* p) { return *p; }

template <typename TIn>
__global__ __launch_bounds__(kBlock) void ingest_row_kernel(const TIn* __restrict__ in,
                                                            float2* __restrict__ out, size_t n) {
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock)
        out[i] = ld_el(in + i);
}

// in [b][A][B] -> out [b][B][A] through a 32x33 LDS tile (element conversion on load).  The
// pitches make it a sub-block transpose: element (a, b) of plane k is in[k*in_plane + a*in_pitch + b]
// and lands at out[k*out_plane + b*out_pitch + a] -- the whole-plane transpose is in_pitch = B,
// out_pitch = A; the host path's pieces use a block of rows or columns of a plane (either side
// may be pinned host memory: the one-CPI calls read their input from, and write their outputs
// into, pinned staging directly).
template <typename TIn, typename TOut>
__global__ __launch_bounds__(kBlock) void transpose_kernel(const TIn* __restrict__ in, TOut* __restrict__ out,
                                                           int A, int B, size_t in_pitch, size_t out_pitch,
                                                           size_t in_plane, size_t out_plane) {
    __shared__ TOut tile[32][33];
    const size_t b = blockIdx.y;
    const int tilesB = (B + 31) / 32;
    const int a0 = (blockIdx.x / tilesB) * 32, b0 = (blockIdx.x % tilesB) * 32;
    const int tx = threadIdx.x % 32, ty = threadIdx.x / 32;
    const TIn* src = in + b * in_plane;
    TOut* dst = out + b * out_plane;
    for (int k = ty; k < 32; k += kBlock / 32) {
        const int aa = a0 + k, bb = b0 + tx;
        if (aa < A && bb < B) tile[k][tx] = ld_el(src + (size_t)aa * in_pitch + bb);
    }
    __syncthreads();
    for (int k = ty; k < 32; k += kBlock / 32) {
        const int bb = b0 + k, aa = a0 + tx;
        if (aa < A && bb < B) dst[(size_t)bb * out_pitch + aa] = tile[tx][k];
    }
}

template <typename TIn, typename TOut>
static hipError_t launch_transpose_t(const TIn* in, TOut* out, int64_t batch, int A, int B, size_t in_pitch,
                                     size_t out_pitch, size_t in_plane, size_t out_plane, hipStream_t s) {
    if (batch <= 0 || A <= 0 || B <= 0) return hipSuccess;
    const unsigned tiles = (unsigned)(((A + 31) / 32) * ((B + 31) / 32));
    for (int64_t b0 = 0; b0 < batch; b0 += 65535) {
        const int64_t nb = batch - b0 < 65535 ? batch - b0 : 65535;
        dim3 grid(tiles, (unsigned)nb), block(kBlock);
        hipLaunchKernelGGL((transpose_kernel<TIn, TOut>), grid, block, 0, s, in + b0 * in_plane, out + b0 * out_plane,
                           A, B, in_pitch, out_pitch, in_plane, out_plane);
    }
    return hipGetLastError();
}
template <typename TIn, typename TOut>
static hipError_t launch_transpose_t(const TIn* in, TOut* out, int64_t batch, int A, int B, hipStream_t s) {
    const size_t plane = (size_t)A * B;
    return launch_transpose_t(in, out, batch, A, B, (size_t)B, (size_t)A, plane, plane, s);
}

hipError_t launch_ingest(const void* in, int dtype, int layout, float2* out, int64_t batch,
                         int P, int R, hipStream_t s) {
    if (layout == RSP_ROWMAJOR) {
        const size_t n = (size_t)batch * P * R;
        if (n == 0) return hipSuccess;
        size_t blocks = (n + kBlock - 1) / kBlock;
        if (blocks > 65536) blocks = 65536;
        dim3 grid((unsigned)blocks), block(kBlock);
        switch (dtype) {
            case RSP_C64: hipLaunchKernelGGL(ingest_row_kernel<float2>, grid, block, 0, s, (const float2*)in, out, n); break;
            case RSP_C128: hipLaunchKernelGGL(ingest_row_kernel<double2>, grid, block, 0, s, (const double2*)in, out, n); break;
            case RSP_C32F16: hipLaunchKernelGGL(ingest_row_kernel<__half2>, grid, block, 0, s, (const __half2*)in, out, n); break;
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    // MATLAB column-major P x R = [b][R][P]  ->  [b][P][R]
    switch (dtype) {
        case RSP_C64: return launch_transpose_t((const float2*)in, out, batch, R, P, s);
        case RSP_C128: return launch_transpose_t((const double2*)in, out, batch, R, P, s);
        case RSP_C32F16: return launch_transpose_t((const __half2*)in, out, batch, R, P, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_transpose_f32(const float* in, float* out, int64_t batch, int A, int B,
                                hipStream_t s) {
    return launch_transpose_t(in, out, batch, A, B, s);
}

hipError_t launch_transpose_u8(const uint8_t* in, uint8_t* out, int64_t batch, int A, int B,
                               hipStream_t s) {
    return launch_transpose_t(in, out, batch, A, B, s);
}

hipError_t launch_transpose_sub(int elem, const void* in, void* out, int A, int B, size_t in_pitch, size_t out_pitch,
                                hipStream_t s) {
    switch (elem) {
        case RSP_SUB_F32:
            return launch_transpose_t((const float*)in, (float*)out, 1, A, B, in_pitch, out_pitch, 0, 0, s);
        case RSP_SUB_U8:
            return launch_transpose_t((const uint8_t*)in, (uint8_t*)out, 1, A, B, in_pitch, out_pitch, 0, 0, s);
        case RSP_SUB_C64:
            return launch_transpose_t((const float2*)in, (float2*)out, 1, A, B, in_pitch, out_pitch, 0, 0, s);
        case RSP_SUB_C32F16:
            return launch_transpose_t((const __half2*)in, (float2*)out, 1, A, B, in_pitch, out_pitch, 0, 0, s);
        default: return hipErrorInvalidValue;
    }
}

// n 4-byte words from `in` to `out` (either may be pinned host memory), 16 bytes per lane
// where both are 16-byte aligned
__global__ __launch_bounds__(kBlock) void copy_words_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                            size_t n) {
    const size_t stride = (size_t)gridDim.x * kBlock;
    const size_t n4 = ((((uintptr_t)in | (uintptr_t)out) & 15u) == 0) ? n / 4 : 0;
    const uint4* in4 = reinterpret_cast<const uint4*>(in);
    uint4* out4 = reinterpret_cast<uint4*>(out);
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n4; i += stride) out4[i] = in4[i];
    for (size_t i = 4 * n4 + blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += stride) out[i] = in[i];
}

hipError_t launch_copy_words(const void* in, void* out, size_t nwords, hipStream_t s) {
    if (nwords == 0) return hipSuccess;
    size_t blocks = (nwords / 4 + kBlock - 1) / kBlock;
    if (blocks < 1) blocks = 1;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(copy_words_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, s, (const uint32_t*)in, (uint32_t*)out,
                       nwords);
    return hipGetLastError();
}

}  // namespace rsp

