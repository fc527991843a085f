// rsp_measure.hip -- post-detection measurement for gfx950: the per-hit
// range / velocity / elevation estimates of motionParaMeasure.m (MatlabProcess_xuzerui/
// CFAR_WangCai/motionParaMeasure.m:1-88, called at DMX_SignalProcessing_main_xzr.m:489-494)
// over a batch of CFAR flag matrices.
//
// One workgroup of 1024 threads per CPI, two passes over the [V][R] flag bytes:
//   count  thread (slice s, column group g) counts the hits of its CW columns in its slice of
//          rows; the counts are laid out in LDS in MATLAB's find() order (column, then row
//          slice) and block-scanned there, which gives every (column, slice) its first output
//          slot without sorting anything;
//   emit   a thread re-reads only the columns it found hits in and measures each hit where it
//          finds it: the 2e+1 cells around it re-anchored as the reference does, a not-a-knot
//          cubic spline through their sum-channel values, its first maximum on the
//          1/interp grid, and the amplitude-ratio elevation.
// The measurement is fp64 with contraction off, in the same operation order as the oracle
// (oracle/measure_ref.py), so the estimates are expected to be bit-identical to it.  The flag
// pass is the HBM traffic (V*R bytes per CPI, read once from HBM, once more from cache for
// the hit columns); the spline work is a few thousand fp64 operations per hit.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/rsp.h"
#include "rsp_internal.h"

namespace rsp {

namespace {

constexpr int kThreads = 1024;

// MATLAB's a:d:b element i of n (colon: first half from a, second half from b).
__device__ __forceinline__ double colon_at(double a, double d, double b, int i, int n) {
#pragma clang fp contract(off)
    return 2 * i < n ? a + (double)i * d : b - (double)(n - 1 - i) * d;
}

// Second derivatives of the not-a-knot cubic spline through y[0..N) at unit-spaced knots
// (oracle/measure_ref.py spline_m).
template <int N>
__device__ __forceinline__ void spline_m(const double (&y)[N], double (&m)[N]) {
#pragma clang fp contract(off)
    if constexpr (N == 3) {
        const double c = y[2] - 2.0 * y[1] + y[0];
        m[0] = c;
        m[1] = c;
        m[2] = c;
    } else {
        double d[N - 2];
#pragma unroll
        for (int i = 1; i < N - 1; ++i) d[i - 1] = 6.0 * (y[i + 1] - 2.0 * y[i] + y[i - 1]);
        m[1] = d[0] / 6.0;
        m[N - 2] = d[N - 3] / 6.0;
        constexpr int K = N - 4;
        if constexpr (K > 0) {
            double rhs[K], c[K], g[K];
#pragma unroll
            for (int i = 0; i < K; ++i) rhs[i] = d[i + 1];
            rhs[0] -= m[1];
            rhs[K - 1] -= m[N - 2];
            c[0] = 1.0 / 4.0;
            g[0] = rhs[0] / 4.0;
#pragma unroll
            for (int i = 1; i < K; ++i) {
                const double den = 4.0 - c[i - 1];
                c[i] = 1.0 / den;
                g[i] = (rhs[i] - g[i - 1]) / den;
            }
            m[2 + K - 1] = g[K - 1];
#pragma unroll
            for (int i = K - 2; i >= 0; --i) m[2 + i] = g[i] - c[i] * m[2 + i + 1];
        }
        m[0] = 2.0 * m[1] - m[2];
        m[N - 1] = 2.0 * m[N - 2] - m[N - 3];
    }
}

// The 1-based cell of the first maximum of the spline through y on cells first..first+N-1,
// sampled at first : 1/interp : first+N-1 (motionParaMeasure.m:36-42, :63-69).
template <int N>
__device__ double refine(const double (&y)[N], int first, int interp) {
#pragma clang fp contract(off)
    double m[N];
    spline_m<N>(y, m);
    const double a = (double)first, b = (double)(first + N - 1);
    const double d = 1.0 / (double)interp;
    const int n = (int)floor((b - a) / d + 1e-10) + 1;
    double best = -INFINITY, qbest = a;
    for (int i = 0; i < n; ++i) {
        const double q = colon_at(a, d, b, i, n);
        const double t = q - a;
        int j = (int)floor(t);
        j = j < 0 ? 0 : (j > N - 2 ? N - 2 : j);
        const double u = t - (double)j, w = 1.0 - u;
        double y0 = y[0], y1 = y[1], m0 = m[0], m1 = m[1];
#pragma unroll
        for (int k = 1; k < N - 1; ++k)   // register select: no dynamic indexing
            if (j == k) {
                y0 = y[k];
                y1 = y[k + 1];
                m0 = m[k];
                m1 = m[k + 1];
            }
        const double v = w * y0 + u * y1 + ((w * w * w - w) * m0 + (u * u * u - u) * m1) / 6.0;
        if (v > best) {
            best = v;
            qbest = q;
        }
    }
    return qbest;
}

// motionParaMeasure.m:22-33 / :49-60: the first of the 2e+1 cells around `center` (1-based),
// moved up to lo or down to hi by anchoring on a member of the set; false where the
// reference's find() comes back empty or the cells leave 1..size (a MATLAB error there).
__device__ __forceinline__ bool fix_cells(int center, int e, int lo, int hi, int size, int* first) {
    int f = center - e;
    if (f < lo) {
        if (lo > f + 2 * e) return false;
        f = lo;
    }
    if (f + 2 * e > hi) {
        if (hi < f) return false;
        f = hi - 2 * e;
    }
    if (f < 1 || f + 2 * e > size) return false;
    *first = f;
    return true;
}

template <int E>
__device__ void measure_hit(const float* __restrict__ sum, const float* __restrict__ diff, int V, int R, int v0,
                            int r0, const MeasureArgs& a, const double* __restrict__ r_scale,
                            const double* __restrict__ v_scale, double* est, bool* bad) {
#pragma clang fp contract(off)
    constexpr int N = 2 * E + 1;
    const int v1 = v0 + 1, r1 = r0 + 1;
    int rf, vf;
    if (!fix_cells(r1, E, 1, R, R, &rf) || !fix_cells(v1, E, a.mtd0_num + 2, V - a.mtd0_num, V, &vf)) {
        est[0] = est[1] = est[2] = NAN;
        *bad = true;
        return;
    }
    double y[N];
#pragma unroll
    for (int k = 0; k < N; ++k) y[k] = (double)sum[(size_t)v0 * R + (rf - 1 + k)];
    const double r_max = refine<N>(y, rf, a.r_interp);
#pragma unroll
    for (int k = 0; k < N; ++k) y[k] = (double)sum[(size_t)(vf - 1 + k) * R + r0];
    const double v_max = refine<N>(y, vf, a.v_interp);
    const double fv = trunc(v_max);
    est[0] = r_scale[r0] + (r_max - (double)r1) * a.delta_r;                        // :43
    est[1] = v_scale[(int)fv - 1] - (v_max - fv) * a.delta_v;                      // :70
    const double ratio = (double)diff[(size_t)v0 * R + r0] / (double)sum[(size_t)v0 * R + r0];   // :78
    est[2] = (double)a.beam_pos_num * a.beam_angle_step + 2.5 - ratio * a.k_value + a.ele_comp + a.ele_sys_err;   // :79
    *bad = false;
}

// Block-wide exclusive scan of one int per thread; returns the thread's prefix, *total the sum.
__device__ __forceinline__ int block_scan(int x, int* s_wave, int* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int inc = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
    }
    if (lane == 63) s_wave[wave] = inc;
    __syncthreads();
    if (threadIdx.x < 64) {
        const int nw = blockDim.x >> 6;
        int w = threadIdx.x < nw ? s_wave[threadIdx.x] : 0;
        int wi = w;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(wi, o, 64);
            if (lane >= o) wi += t;
        }
        if (threadIdx.x < nw) s_wave[threadIdx.x] = wi - w;   // exclusive wave prefix
        if (threadIdx.x == nw - 1) s_wave[32] = wi;
    }
    __syncthreads();
    const int r = s_wave[wave] + inc - x;
    *total = s_wave[32];
    __syncthreads();   // s_wave is reused by the next call
    return r;
}

// CW columns per thread (4: one 32-bit load per row when R % 4 == 0), G column groups and
// S = 1024 / G row slices per pass.
template <int E, int CW>
__global__ __launch_bounds__(kThreads) void measure_kernel(const float* __restrict__ sum, const float* __restrict__ diff,
                                                           const uint8_t* __restrict__ flag, int V, int R, int G,
                                                           MeasureArgs a, const double* __restrict__ r_scale,
                                                           const double* __restrict__ v_scale, int64_t max_hits,
                                                           double* __restrict__ est, int32_t* __restrict__ cells,
                                                           int32_t* __restrict__ count) {
    __shared__ int s_cnt[kThreads * CW];
    __shared__ int s_wave[33];
    __shared__ int s_bad;
    const int cpi = blockIdx.x;
    const size_t plane = (size_t)V * R;
    const uint8_t* fl = flag + cpi * plane;
    const float* su = sum + cpi * plane;
    const float* di = diff + cpi * plane;
    double* es = est + (size_t)cpi * max_hits * 3;
    int32_t* ce = cells ? cells + (size_t)cpi * max_hits * 2 : nullptr;
    const int S = kThreads / G;
    const int g = threadIdx.x % G, s = threadIdx.x / G;
    const int rows = (V + S - 1) / S;
    const int v_lo = s * rows, v_hi = min(V, v_lo + rows);
    if (threadIdx.x == 0) s_bad = 0;
    int base = 0;   // hits of the earlier column passes
    for (int c_pass = 0; c_pass < R; c_pass += G * CW) {
        const int c0 = c_pass + g * CW;
        int cnt[CW];
#pragma unroll
        for (int j = 0; j < CW; ++j) cnt[j] = 0;
        if (c0 < R) {
            if constexpr (CW == 4) {
#pragma unroll 8
                for (int v = v_lo; v < v_hi; ++v) {
                    const uint32_t w = *reinterpret_cast<const uint32_t*>(fl + (size_t)v * R + c0);
#pragma unroll
                    for (int j = 0; j < 4; ++j) cnt[j] += (w >> (8 * j)) & 0xffu ? 1 : 0;
                }
            } else {
#pragma unroll 8
                for (int v = v_lo; v < v_hi; ++v) cnt[0] += fl[(size_t)v * R + c0] ? 1 : 0;
            }
        }
        // counts in find() order: column c_pass + k (k = g*CW + j), then row slice s
#pragma unroll
        for (int j = 0; j < CW; ++j) s_cnt[(g * CW + j) * S + s] = cnt[j];
        __syncthreads();
        int run[CW], mine = 0;
#pragma unroll
        for (int j = 0; j < CW; ++j) {
            run[j] = s_cnt[threadIdx.x * CW + j];
            mine += run[j];
        }
        int total;
        int pre = block_scan(mine, s_wave, &total);
#pragma unroll
        for (int j = 0; j < CW; ++j) {
            const int x = run[j];
            s_cnt[threadIdx.x * CW + j] = base + pre;
            pre += x;
        }
        __syncthreads();
        // emit: re-read the columns with hits, measure each hit in its slot
#pragma unroll
        for (int j = 0; j < CW; ++j) {
            if (cnt[j] == 0) continue;
            const int c = c0 + j;
            int slot = s_cnt[(g * CW + j) * S + s];
            int left = cnt[j];
            for (int v = v_lo; v < v_hi && left > 0; ++v) {
                if (!fl[(size_t)v * R + c]) continue;
                --left;
                if (slot < max_hits) {
                    double e3[3];
                    bool bad;
                    measure_hit<E>(su, di, V, R, v, c, a, r_scale, v_scale, e3, &bad);
                    es[(size_t)slot * 3 + 0] = e3[0];
                    es[(size_t)slot * 3 + 1] = e3[1];
                    es[(size_t)slot * 3 + 2] = e3[2];
                    if (ce) {
                        ce[(size_t)slot * 2 + 0] = v;
                        ce[(size_t)slot * 2 + 1] = c;
                    }
                    if (bad) atomicAdd(&s_bad, 1);
                } else {   // counted, not written: only whether the reference would stop here
                    int f0;
                    if (!fix_cells(c + 1, E, 1, R, R, &f0) || !fix_cells(v + 1, E, a.mtd0_num + 2, V - a.mtd0_num, V, &f0))
                        atomicAdd(&s_bad, 1);
                }
                ++slot;
            }
        }
        base += total;
        __syncthreads();   // s_cnt is rewritten by the next pass
    }
    if (threadIdx.x == 0) {
        count[cpi * 2 + 0] = base;
        count[cpi * 2 + 1] = s_bad;
    }
}

template <int E>
hipError_t launch_e(const float* sum, const float* diff, const uint8_t* flag, int V, int R, int batch,
                    const MeasureArgs& a, const double* r_scale, const double* v_scale, int64_t max_hits,
                    double* est, int32_t* cells, int32_t* count, hipStream_t st) {
    const bool wide = R % 4 == 0 && R >= 4 * 64 && ((uintptr_t)flag & 3) == 0;
    int G = 64;   // column groups per pass: a power of two covering the columns, at most 1024
    const int groups = wide ? R / 4 : R;
    while (G < groups && G < kThreads) G <<= 1;
    if (wide)
        hipLaunchKernelGGL((measure_kernel<E, 4>), dim3(batch), dim3(kThreads), 0, st, sum, diff, flag, V, R, G, a,
                           r_scale, v_scale, max_hits, est, cells, count);
    else
        hipLaunchKernelGGL((measure_kernel<E, 1>), dim3(batch), dim3(kThreads), 0, st, sum, diff, flag, V, R, G, a,
                           r_scale, v_scale, max_hits, est, cells, count);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_measure(const float* sum, const float* diff, const uint8_t* flag, int V, int R, int batch,
                          const MeasureArgs& a, const double* r_scale, const double* v_scale, int64_t max_hits,
                          double* est, int32_t* cells, int32_t* count, hipStream_t st) {
    if (batch <= 0) return hipSuccess;
    switch (a.extra_dots) {
        case 1: return launch_e<1>(sum, diff, flag, V, R, batch, a, r_scale, v_scale, max_hits, est, cells, count, st);
        case 2: return launch_e<2>(sum, diff, flag, V, R, batch, a, r_scale, v_scale, max_hits, est, cells, count, st);
        case 3: return launch_e<3>(sum, diff, flag, V, R, batch, a, r_scale, v_scale, max_hits, est, cells, count, st);
        case 4: return launch_e<4>(sum, diff, flag, V, R, batch, a, r_scale, v_scale, max_hits, est, cells, count, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace rsp
