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

#include "rsp_fft.h"
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
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)pc_kernel<float2>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e == hipSuccess)
            e = hipFuncSetAttribute((const void*)pc_kernel<__half2>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
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
    static constexpr int G = N / 16;                            // threads per row
    static constexpr int E = N / G;                             // 16 elements per thread
    static constexpr int RPB = G >= 256 ? 1 : 256 / G;          // rows per workgroup
    static constexpr int T = G * RPB;
    static constexpr int SLOT = padded_len(N);
    static constexpr size_t lds = (size_t)RPB * SLOT * sizeof(float2);
};

template <typename TIn, int G>
__device__ __forceinline__ void fir_row(const TIn* __restrict__ x, float2* __restrict__ y,
                                        const SegDev& g, float* stage, bool valid, int t) {
    // stage the segment's input, then y[n] = scale * sum_k taps[k] x[m-k], m = (n+shift) mod len
    float2* s2 = reinterpret_cast<float2*>(stage);
    for (int i = t; i < g.in_len; i += G) s2[i] = valid ? ld_c(x + g.in_start + i) : make_float2(0.f, 0.f);
    __syncthreads();
    for (int n = t; n < g.out_len; n += G) {
        int m = n + g.fir_shift;
        if (m >= g.out_len) m -= g.out_len;
        float ar = 0.f, ai = 0.f;
        const int kmax = m + 1 < g.ntaps ? m + 1 : g.ntaps;
        const float* __restrict__ taps = g.taps_dev;
        for (int k = 0; k < kmax; ++k) {
            const float2 v = s2[m - k];
            const float b = taps[k];
            ar = fmaf(b, v.x, ar);
            ai = fmaf(b, v.y, ai);
        }
        if (valid) y[g.out_start + n] = make_float2(ar * g.scale, ai * g.scale);
    }
    __syncthreads();
}

// One row's matched-filter segment (and optionally its FIR segment) by G threads.
template <typename TIn, int N, int G>
__device__ __forceinline__ void pc_row(const TIn* __restrict__ echo, float2* __restrict__ out,
                                       const PcMfArgs& a, int row, int t, float2* buf) {
    constexpr int E = N / G;
    const bool valid = row < a.rows;
    const TIn* x = echo + (size_t)row * a.R;
    float2* y = out + (size_t)row * a.R_out;
    if (a.do_fir) {
        if (valid)
            for (int z = 0; z < a.nzero; ++z)
                for (int c = a.zero_lo[z] + t; c < a.zero_hi[z]; c += G) y[c] = make_float2(0.f, 0.f);
        fir_row<TIn, G>(x, y, a.fir, reinterpret_cast<float*>(buf), valid, t);
    }
    const int in_start = a.mf.in_start, in_len = a.mf.in_len;
    const int out_start = a.mf.out_start, out_len = a.mf.out_len;
    const float2* __restrict__ H = a.mf.H;
    const float2* __restrict__ tw = a.mf.tw;
    float2 u[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const int i = t + G * m;
        u[m] = (valid && i < in_len) ? ld_c(x + in_start + i) : make_float2(0.f, 0.f);
    }
    fft_reg<N, G, 1, E>(u, buf, t, tw);
#pragma unroll
    for (int m = 0; m < E; ++m) u[m] = cconj(cmul(u[m], H[t + G * m]));  // conj(X.*H), 1/N in H
    fft_reg<N, G, 1, E>(u, buf, t, tw);
    if (valid) {
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int i = t + G * m;
            if (i < out_len) y[out_start + i] = cconj(u[m]);
        }
    }
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
template <typename TIn, int N1, int N2>
__global__ __launch_bounds__((PairCfg<N1, (N2 ? N2 : N1)>::T), 4) void pc_mf_kernel(
    const TIn* __restrict__ echo, float2* __restrict__ out, PcMfArgs a1, PcMfArgs a2, int nblk2) {
    constexpr int M2 = N2 ? N2 : N1;
    using PC = PairCfg<N1, M2>;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    if constexpr (N2 != 0) {
        if ((int)blockIdx.x < nblk2) {
            constexpr int G = PcCfg<N2>::G;
            const int grp = threadIdx.x / G, t = threadIdx.x % G;
            pc_row<TIn, N2, G>(echo, out, a2, blockIdx.x * PC::RPB2 + grp, t, lds + grp * PcCfg<N2>::SLOT);
            return;
        }
    }
    constexpr int G = PcCfg<N1>::G;
    const int grp = threadIdx.x / G, t = threadIdx.x % G;
    const int b = (int)blockIdx.x - (N2 ? nblk2 : 0);
    pc_row<TIn, N1, G>(echo, out, a1, b * PC::RPB1 + grp, t, lds + grp * PcCfg<N1>::SLOT);
}

bool pc_mf_supported(int nfft, int fir_in_len) {
    switch (nfft) {
        case 64: case 128: case 256: case 512: case 1024: case 2048: case 4096: case 8192:
        case 16384:
            return fir_in_len <= padded_len(nfft);   // the FIR stages its input in the row's slot
        default:
            return false;
    }
}

template <typename TIn, int N1, int N2>
static hipError_t launch_pc_mf_n(const TIn* echo, float2* out, const PcMfArgs& a1, const PcMfArgs* a2,
                                 hipStream_t s) {
    constexpr int M2 = N2 ? N2 : N1;
    using PC = PairCfg<N1, M2>;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)pc_mf_kernel<TIn, N1, N2>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)PC::lds);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    const int nblk1 = (a1.rows + PC::RPB1 - 1) / PC::RPB1;
    const int nblk2 = N2 ? (a1.rows + PC::RPB2 - 1) / PC::RPB2 : 0;
    dim3 grid((unsigned)(nblk1 + nblk2)), block(PC::T);
    hipLaunchKernelGGL((pc_mf_kernel<TIn, N1, N2>), grid, block, PC::lds, s, echo, out, a1,
                       a2 ? *a2 : a1, nblk2);
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

// ================================================================== Doppler CFAR (column tile)
// mag: W columns of V floats, column stride ms; flags written to out[v*R + r0 + c].
__device__ __forceinline__ void doppler_cfar_tile(const float* mag, int ms, int V, int W,
                                                  const CfarVArgs& cv, uint8_t* __restrict__ out,
                                                  int r0, int R, int t) {
    for (int e = t; e < V * W; e += kBlock) {
        const int c = e % W, v = e / W, r = r0 + c;
        if (r >= R) continue;
        bool in_seg = false;
        for (int s = 0; s < cv.nseg; ++s) in_seg |= (r >= cv.seg_lo[s] && r < cv.seg_hi[s]);
        uint8_t f = 0;
        if (in_seg && v >= cv.lo && v < cv.hi) {
            const float* col = mag + c * ms;
            const int l1 = v - cv.save - cv.ref;  // left window [l1, v-save-1]
            const int r1 = v + cv.save + 1;       // right window [r1, v+save+ref]
            const bool lok = l1 >= cv.lo;
            const bool rok = r1 + cv.ref - 1 < cv.hi;
            float sl = 0.f, sr = 0.f;
            if (lok)
                for (int i = 0; i < cv.ref; ++i) sl += col[l1 + i];
            if (rok)
                for (int i = 0; i < cv.ref; ++i) sr += col[r1 + i];
            const float lavg = (lok ? sl : sr) / (float)cv.ref;   // mean() of 5 cells
            const float ravg = (rok ? sr : sl) / (float)cv.ref;
            const float avg = cv.method == 0 ? fmaxf(lavg, ravg) : fminf(lavg, ravg);
            f = col[v] >= avg * cv.T ? 1 : 0;
        }
        out[(size_t)v * R + r] = f;
    }
}

// ================================================================== MTD (+ Doppler CFAR)
__host__ __device__ constexpr int pow2floor(int x) {
    int p = 1;
    while (p * 2 <= x) p *= 2;
    return p;
}

template <int P>
struct MtdCfg {
    static constexpr int G = (P / 16) < 1 ? 1 : ((P / 16) >= 64 ? 64 : pow2floor(P / 16));
    static constexpr int W = kBlock / G;           // range bins per workgroup
    static constexpr int CS = padded_len(P);       // float2 stride of one column
    static constexpr int MS = P + 1;               // float stride of one magnitude column
    static constexpr size_t lds = (size_t)W * CS * sizeof(float2) + (size_t)W * MS * sizeof(float);
};

template <int P>
__global__ __launch_bounds__(kBlock) void mtd_kernel(const float2* __restrict__ pc,
                                                     float* __restrict__ rdm,
                                                     uint8_t* __restrict__ flagV, MtdArgs a) {
    using C = MtdCfg<P>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float2* cbuf = reinterpret_cast<float2*>(smem);
    float* mag = reinterpret_cast<float*>(smem + (size_t)C::W * C::CS * sizeof(float2));
    const int t = threadIdx.x;
    const size_t cpi = blockIdx.y;
    const int r0 = blockIdx.x * C::W;
    const int R = a.R_out;
    const float2* src = pc + cpi * (size_t)P * R;

    for (int e = t; e < P * C::W; e += kBlock) {
        const int c = e % C::W, p = e / C::W, r = r0 + c;
        float2 v = make_float2(0.f, 0.f);
        if (r < R) v = src[(size_t)p * R + r];
        const float w = a.win[p];
        cbuf[c * C::CS + pidx(p)] = make_float2(v.x * w, v.y * w);
    }
    __syncthreads();
    fft_lds<P, C::G>(cbuf + (t / C::G) * C::CS, t % C::G, a.tw);

    float* dst = rdm + cpi * (size_t)P * R;
    const bool cfar = a.cv.enabled != 0;
    for (int e = t; e < P * C::W; e += kBlock) {
        const int c = e % C::W, v = e / C::W, r = r0 + c;
        int q = v - a.shift;
        if (q < 0) q += P;
        const float2 X = cbuf[c * C::CS + pidx(q)];
        float m = sqrtf(fmaf(X.x, X.x, X.y * X.y));
        if (v >= a.z_lo && v < a.z_hi) m = 0.f;
        if (r < R) dst[(size_t)v * R + r] = m;
        if (cfar) mag[c * C::MS + v] = (v >= a.cv.cz_lo && v < a.cv.cz_hi) ? 0.f : m;
    }
    if (cfar) {
        __syncthreads();
        doppler_cfar_tile(mag, C::MS, P, C::W, a.cv, flagV + cpi * (size_t)P * R, r0, R, t);
    }
}

template <int P>
static hipError_t launch_mtd_p(const float2* pc, float* rdm, uint8_t* flagV, int ncpi,
                               const MtdArgs& a, hipStream_t s) {
    using C = MtdCfg<P>;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)mtd_kernel<P>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)C::lds);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    dim3 grid((unsigned)((a.R_out + C::W - 1) / C::W), (unsigned)ncpi), block(kBlock);
    hipLaunchKernelGGL(mtd_kernel<P>, grid, block, C::lds, s, pc, rdm, flagV, a);
    return hipGetLastError();
}

bool mtd_size_supported(int P) {
    switch (P) {
        case 16: case 32: case 64: case 128: case 256: case 512: case 1024:
        case 48: case 96: case 192: case 384: case 768: case 1536:
            return true;
        default:
            return false;
    }
}

hipError_t launch_mtd(const float2* pc, float* rdm, uint8_t* flagV, int ncpi, const MtdArgs& a,
                      hipStream_t s) {
    if (ncpi <= 0) return hipSuccess;
    switch (a.P) {
        case 16: return launch_mtd_p<16>(pc, rdm, flagV, ncpi, a, s);
        case 32: return launch_mtd_p<32>(pc, rdm, flagV, ncpi, a, s);
        case 64: return launch_mtd_p<64>(pc, rdm, flagV, ncpi, a, s);
        case 128: return launch_mtd_p<128>(pc, rdm, flagV, ncpi, a, s);
        case 256: return launch_mtd_p<256>(pc, rdm, flagV, ncpi, a, s);
        case 512: return launch_mtd_p<512>(pc, rdm, flagV, ncpi, a, s);
        case 1024: return launch_mtd_p<1024>(pc, rdm, flagV, ncpi, a, s);
        case 48: return launch_mtd_p<48>(pc, rdm, flagV, ncpi, a, s);
        case 96: return launch_mtd_p<96>(pc, rdm, flagV, ncpi, a, s);
        case 192: return launch_mtd_p<192>(pc, rdm, flagV, ncpi, a, s);
        case 384: return launch_mtd_p<384>(pc, rdm, flagV, ncpi, a, s);
        case 768: return launch_mtd_p<768>(pc, rdm, flagV, ncpi, a, s);
        case 1536: return launch_mtd_p<1536>(pc, rdm, flagV, ncpi, a, s);
        default: return hipErrorInvalidValue;
    }
}

// ================================================================== Doppler CFAR from an RDM
__global__ __launch_bounds__(kBlock) void cfar_v_kernel(const float* __restrict__ rdm,
                                                        uint8_t* __restrict__ flagV, int V, int R,
                                                        int W, CfarVArgs cv) {
    extern __shared__ __attribute__((aligned(16))) float magv[];
    const int t = threadIdx.x;
    const size_t cpi = blockIdx.y;
    const int r0 = blockIdx.x * W;
    const int ms = V + 1;
    const float* src = rdm + cpi * (size_t)V * R;
    for (int e = t; e < V * W; e += kBlock) {
        const int c = e % W, v = e / W, r = r0 + c;
        float m = 0.f;
        if (r < R && !(v >= cv.cz_lo && v < cv.cz_hi)) m = src[(size_t)v * R + r];
        magv[c * ms + v] = m;
    }
    __syncthreads();
    doppler_cfar_tile(magv, ms, V, W, cv, flagV + cpi * (size_t)V * R, r0, R, t);
}

hipError_t launch_cfar_v(const float* rdm, uint8_t* flagV, int ncpi, int V, int R,
                         const CfarVArgs& a, hipStream_t s) {
    if (ncpi <= 0) return hipSuccess;
    int W = 64;
    while (W > 1 && (size_t)W * (V + 1) * sizeof(float) > 64 * 1024) W /= 2;
    const size_t lds = (size_t)W * (V + 1) * sizeof(float);
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)cfar_v_kernel,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    dim3 grid((unsigned)((R + W - 1) / W), (unsigned)ncpi), block(kBlock);
    hipLaunchKernelGGL(cfar_v_kernel, grid, block, lds, s, rdm, flagV, V, R, W, a);
    return hipGetLastError();
}

// ================================================================== range CFAR + re-localisation
__global__ __launch_bounds__(kBlock) void cfar_r_kernel(const float* __restrict__ rdm,
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
    float* x = reinterpret_cast<float*>(smem);
    uint8_t* fv = smem + (size_t)R * sizeof(float);
    uint8_t* pass = fv + R;
    const bool zrow = (v >= a.cz_lo && v < a.cz_hi);
    const float* xr = rdm + rowoff;
    for (int c = t; c < R; c += kBlock) {
        x[c] = zrow ? 0.f : xr[c];
        fv[c] = fv_g[c];
    }
    __syncthreads();
    for (int c = t; c < R; c += kBlock) {
        int slo = 0, shi = 0;
        for (int s = 0; s < a.nseg; ++s)
            if (c >= a.seg_lo[s] && c < a.seg_hi[s]) { slo = a.seg_lo[s]; shi = a.seg_hi[s]; }
        uint8_t p = 0;
        if (shi > slo) {
            const int l1 = c - a.save - a.ref;
            const int r1 = c + a.save + 1;
            const bool lok = l1 >= slo;
            const bool rok = r1 + a.ref - 1 < shi;
            float sl = 0.f, sr = 0.f;
            if (lok)
                for (int i = 0; i < a.ref; ++i) sl += x[l1 + i];
            if (rok)
                for (int i = 0; i < a.ref; ++i) sr += x[r1 + i];
            const float lavg = (lok ? sl : sr) / (float)a.ref;
            const float ravg = (rok ? sr : sl) / (float)a.ref;
            const float avg = a.method == 0 ? fmaxf(lavg, ravg) : fminf(lavg, ravg);
            p = x[c] >= avg * a.T ? 1 : 0;
        }
        pass[c] = p;
    }
    __syncthreads();
    for (int c = t; c < R; c += kBlock) {
        int slo = 0, shi = 0;
        for (int s = 0; s < a.nseg; ++s)
            if (c >= a.seg_lo[s] && c < a.seg_hi[s]) { slo = a.seg_lo[s]; shi = a.seg_hi[s]; }
        uint8_t f = 0;
        for (int d = -1; d <= 1 && shi > slo; ++d) {
            const int r = c + d;  // a Doppler hit at r tests cells r-1..r+1
            if (r < slo || r >= shi || !fv[r]) continue;
            int best = -1;
            float bx = 0.f;
            for (int e2 = -1; e2 <= 1; ++e2) {
                const int q = r + e2;
                if (q < slo || q >= shi || !pass[q]) continue;
                if (best < 0 || x[q] > bx) { best = q; bx = x[q]; }  // first max
            }
            if (best == c) f = 1;
        }
        out[c] = f;
    }
}

hipError_t launch_cfar_r(const float* rdm, const uint8_t* flagV, uint8_t* flag, int ncpi,
                         const CfarRArgs& a, hipStream_t s) {
    if (ncpi <= 0) return hipSuccess;
    const size_t lds = (size_t)a.R * (sizeof(float) + 2);
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)cfar_r_kernel,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    dim3 grid((unsigned)a.V, (unsigned)ncpi), block(kBlock);
    hipLaunchKernelGGL(cfar_r_kernel, grid, block, lds, s, rdm, flagV, flag, a);
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

// in [b][A][B] -> out [b][B][A] through a 32x33 LDS tile (element conversion on load)
template <typename TIn, typename TOut>
__global__ __launch_bounds__(kBlock) void transpose_kernel(const TIn* __restrict__ in,
                                                           TOut* __restrict__ out, int A, int B) {
    __shared__ TOut tile[32][33];
    const size_t b = blockIdx.y;
    const int tilesB = (B + 31) / 32;
    const int a0 = (blockIdx.x / tilesB) * 32, b0 = (blockIdx.x % tilesB) * 32;
    const int tx = threadIdx.x % 32, ty = threadIdx.x / 32;
    const TIn* src = in + b * (size_t)A * B;
    TOut* dst = out + b * (size_t)A * B;
    for (int k = ty; k < 32; k += kBlock / 32) {
        const int aa = a0 + k, bb = b0 + tx;
        if (aa < A && bb < B) tile[k][tx] = ld_el(src + (size_t)aa * B + bb);
    }
    __syncthreads();
    for (int k = ty; k < 32; k += kBlock / 32) {
        const int bb = b0 + k, aa = a0 + tx;
        if (aa < A && bb < B) dst[(size_t)bb * A + aa] = tile[tx][k];
    }
}

template <typename TIn, typename TOut>
static hipError_t launch_transpose_t(const TIn* in, TOut* out, int64_t batch, int A, int B,
                                     hipStream_t s) {
    if (batch <= 0 || A <= 0 || B <= 0) return hipSuccess;
    const unsigned tiles = (unsigned)(((A + 31) / 32) * ((B + 31) / 32));
    for (int64_t b0 = 0; b0 < batch; b0 += 65535) {
        const int64_t nb = batch - b0 < 65535 ? batch - b0 : 65535;
        dim3 grid(tiles, (unsigned)nb), block(kBlock);
        hipLaunchKernelGGL((transpose_kernel<TIn, TOut>), grid, block, 0, s,
                           in + b0 * (size_t)A * B, out + b0 * (size_t)A * B, A, B);
    }
    return hipGetLastError();
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

}  // namespace rsp
