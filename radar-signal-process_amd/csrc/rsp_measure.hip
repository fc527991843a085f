// rsp_measure.hip -- post-detection measurement for gfx950: the per-hit
// range / velocity / elevation estimates of motionParaMeasure.m (MatlabProcess_xuzerui/
// CFAR_WangCai/motionParaMeasure.m:1-88, called at DMX_SignalProcessing_main_xzr.m:489-494)
// over a batch of CFAR flag matrices.
//
// Two launches:
//   hits_kernel     one workgroup of 1024 threads per CPI, two passes over the [V][R] flag
//                   bytes.  count: thread (slice s, column group g) counts the hits of its CW
//                   columns in its slice of rows; the counts are laid out in LDS in MATLAB's
//                   find() order (column, then row slice) and block-scanned there, which gives
//                   every (column, slice) its first output slot without sorting anything.
//                   The count pass also keeps a 64-bit mask of which of the thread's row
//                   groups hold hits; list: a thread re-reads only those rows and writes each
//                   hit's cell index into its slot.
//   measure_kernel  one thread per listed hit over the whole batch: the 2e+1 cells around it
//                   re-anchored as the reference does, a not-a-knot cubic spline through their
//                   sum-channel values, its first maximum on the 1/interp grid, and the
//                   amplitude-ratio elevation.  Spreading hits over the chip (instead of
//                   measuring them inside the CPI's workgroup) keeps the per-hit dependent
//                   loads and fp64 work off the flag scan's critical path.
// The measurement is fp64 with contraction off, in the same operation order as the oracle
// (oracle/measure_ref.py), so the estimates are bit-identical to it.  The flag scan is the
// HBM traffic (V*R bytes per CPI, read once from HBM, once more from cache for the rows with
// hits); the spline work is a few thousand fp64 operations per hit.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

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
// sampled at first : 1/interp : first+N-1 (motionParaMeasure.m:36-42, :63-69).  Each interval
// j is evaluated in Horner form y_j + u*(b_j + u*(c_j + u*d_j)) (oracle/measure_ref.py
// spline_eval); the samples are walked interval by interval (their abscissae are increasing),
// so every coefficient stays in a register.
template <int N>
__device__ double refine(const double (&y)[N], int first, int interp) {
#pragma clang fp contract(off)
    double m[N];
    spline_m<N>(y, m);
    double cb[N - 1], cc[N - 1], cd[N - 1];
#pragma unroll
    for (int j = 0; j < N - 1; ++j) {
        cb[j] = (y[j + 1] - y[j]) - (2.0 * m[j] + m[j + 1]) / 6.0;
        cc[j] = m[j] / 2.0;
        cd[j] = (m[j + 1] - m[j]) / 6.0;
    }
    const double a = (double)first, b = (double)(first + N - 1);
    const double d = 1.0 / (double)interp;
    const int n = (int)floor((b - a) / d + 1e-10) + 1;
    double best = -INFINITY, qbest = a;
    int i = 0;
#pragma unroll
    for (int j = 0; j < N - 1; ++j) {
        for (; i < n; ++i) {
            const double q = colon_at(a, d, b, i, n);
            const double t = q - a;
            int jj = (int)floor(t);
            jj = jj < 0 ? 0 : (jj > N - 2 ? N - 2 : jj);
            if (jj > j) break;
            const double u = t - (double)j;
            const double v = y[j] + u * (cb[j] + u * (cc[j] + u * cd[j]));
            if (v > best) {
                best = v;
                qbest = q;
            }
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
    // every load up front (one round of latency): the range and velocity cells, the hit's
    // sum / diff, rScale(r) and the N vScale entries fix(vCellMax) can select
    float fr[N], fvv[N];
    double vs[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
        fr[k] = sum[(size_t)v0 * a.ld + (rf - 1 + k)];
        fvv[k] = sum[(size_t)(vf - 1 + k) * a.ld + r0];
        vs[k] = v_scale[vf - 1 + k];
    }
    const float s_hit = sum[(size_t)v0 * a.ld + r0], d_hit = diff[(size_t)v0 * a.ld + r0];
    const double rs = r_scale[r0];
    double y[N];
#pragma unroll
    for (int k = 0; k < N; ++k) y[k] = (double)fr[k];
    const double r_max = refine<N>(y, rf, a.r_interp);
#pragma unroll
    for (int k = 0; k < N; ++k) y[k] = (double)fvv[k];
    const double v_max = refine<N>(y, vf, a.v_interp);
    const double fv = trunc(v_max);
    const int kv = (int)fv - vf;   // 0..N-1: v_max lies in [vf, vf+N-1]
    double vsel = vs[0];
#pragma unroll
    for (int k = 1; k < N; ++k)
        if (kv == k) vsel = vs[k];
    est[0] = rs + (r_max - (double)r1) * a.delta_r;                                  // :43
    est[1] = vsel - (v_max - fv) * a.delta_v;                                        // :70
    const double ratio = (double)d_hit / (double)s_hit;                              // :78
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

// Bit j set where flag byte j of the CW at fl[v*R + c0] is nonzero (CW = 16: one 16-byte load).
template <int CW>
__device__ __forceinline__ uint32_t row_pattern(const uint8_t* __restrict__ fl, size_t off) {
    if constexpr (CW == 16) {
        const uint4 w = *reinterpret_cast<const uint4*>(fl + off);
        const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
        uint32_t pat = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            // high bit of each byte = byte nonzero
            const uint32_t t = (((ws[k] & 0x7f7f7f7fu) + 0x7f7f7f7fu) | ws[k]) & 0x80808080u;
            pat |= (((t >> 7) & 1u) | ((t >> 14) & 2u) | ((t >> 21) & 4u) | ((t >> 28) & 8u)) << (4 * k);
        }
        return pat;
    } else {
        return fl[off] ? 1u : 0u;
    }
}

// CW columns per thread (16: one 16-byte load per row when R % 16 == 0), G column groups and
// S = 1024 / G row slices per pass; each thread owns `rows` rows of its CW columns.
template <int E, int CW>
__global__ __launch_bounds__(kThreads) void hits_kernel(const uint8_t* __restrict__ flag, int V, int R, int G,
                                                        int64_t ld, int64_t cs, int mtd0_num, int64_t max_hits, double* __restrict__ est,
                                                        int32_t* __restrict__ count) {
    __shared__ int s_cnt[kThreads * CW];
    __shared__ int s_wave[33];
    __shared__ int s_bad;
    const int cpi = blockIdx.x;
    const uint8_t* fl = flag + cpi * cs;
    int64_t* hl = reinterpret_cast<int64_t*>(est) + (size_t)cpi * max_hits * 3;   // hit list, slot * 3
    const int S = kThreads / G;
    const int g = threadIdx.x % G, s = threadIdx.x / G;
    const int rows = (V + S - 1) / S;
    const int v_lo = min(V, s * rows), v_hi = min(V, v_lo + rows);
    const int q = (rows + 63) / 64;   // rows per bit of the thread's row mask
    if (threadIdx.x == 0) s_bad = 0;
    int base = 0;   // hits of the earlier column passes
    for (int c_pass = 0; c_pass < R; c_pass += G * CW) {
        const int c0 = c_pass + g * CW;
        int cnt[CW];
#pragma unroll
        for (int j = 0; j < CW; ++j) cnt[j] = 0;
        uint64_t rmask = 0;   // bit i: rows v_lo + i*q .. + q-1 hold a hit
        if (c0 < R) {
#pragma unroll 8
            for (int v = v_lo; v < v_hi; ++v) {
                const uint32_t pat = row_pattern<CW>(fl, (size_t)v * ld + c0);
#pragma unroll
                for (int j = 0; j < CW; ++j) cnt[j] += (pat >> j) & 1u;
                rmask |= (uint64_t)(pat != 0) << ((v - v_lo) / q);
            }
        }
        // counts in find() order: column c_pass + k (k = g*CW + j), then row slice s
#pragma unroll
        for (int j = 0; j < CW; ++j) s_cnt[(g * CW + j) * S + s] = cnt[j];
        __syncthreads();
        int run[CW], part = 0;
#pragma unroll
        for (int j = 0; j < CW; ++j) {
            run[j] = s_cnt[threadIdx.x * CW + j];
            part += run[j];
        }
        int total;
        int pre = block_scan(part, s_wave, &total);
#pragma unroll
        for (int j = 0; j < CW; ++j) {
            const int x = run[j];
            s_cnt[threadIdx.x * CW + j] = base + pre;
            pre += x;
        }
        __syncthreads();
        // list: re-read only the row groups the mask marks (ascending rows), and give each hit
        // its column's next slot; each (column, slice) keeps its next slot in its own LDS word,
        // so the order is find()'s.
        while (rmask) {
            const int i = __builtin_ctzll(rmask);
            rmask &= rmask - 1;
            const int r_hi = min(v_hi, v_lo + (i + 1) * q);
            for (int v = v_lo + i * q; v < r_hi; ++v) {
                uint32_t pat = row_pattern<CW>(fl, (size_t)v * ld + c0);
                while (pat) {
                    const int j = __builtin_ctz(pat);
                    pat &= pat - 1;
                    const int c = c0 + j;
                    int* nx = &s_cnt[(g * CW + j) * S + s];
                    const int slot = *nx;
                    *nx = slot + 1;
                    if (slot < max_hits) {
                        hl[(size_t)slot * 3] = (int64_t)v * R + c;   // measured by measure_kernel
                    } else {   // counted, not written: only whether the reference would stop here
                        int f0;
                        if (!fix_cells(c + 1, E, 1, R, R, &f0) ||
                            !fix_cells(v + 1, E, mtd0_num + 2, V - mtd0_num, V, &f0))
                            atomicAdd(&s_bad, 1);
                    }
                }
            }
        }
        base += total;
        __syncthreads();   // s_cnt is rewritten by the next pass
    }
    if (threadIdx.x == 0) {
        count[cpi * 2 + 0] = base;
        count[cpi * 2 + 1] = s_bad;   // measure_kernel adds the written hits' failures
    }
}

// ---- banded hit lists (opt-in, see measure_bands): several workgroups per CPI, each owning
// a band of Vb rows, in three launches -- band counts per column, one scan per CPI in find()
// order (column, then band), band lists with those offsets -- meant for batches below the CU
// count, where one workgroup per CPI leaves most of the chip idle.

// Per-column hit counts of band `band`: cnt[(cpi * R + c) * nb + band] (scan order).
template <int CW>
__global__ __launch_bounds__(kThreads) void band_count_kernel(const uint8_t* __restrict__ flag, int V, int R, int G,
                                                              int64_t ld, int64_t cs, int nb, int Vb,
                                                              int32_t* __restrict__ cnt) {
    __shared__ int s_cnt[kThreads * CW];
    const int cpi = blockIdx.x / nb, band = blockIdx.x - cpi * nb;
    const uint8_t* fl = flag + cpi * cs;
    const int S = kThreads / G;
    const int g = threadIdx.x % G, s = threadIdx.x / G;
    const int b_lo = band * Vb, b_hi = min(V, b_lo + Vb);
    const int rows = (b_hi - b_lo + S - 1) / S;
    const int v_lo = min(b_hi, b_lo + s * rows), v_hi = min(b_hi, v_lo + rows);
    int32_t* out = cnt + (size_t)cpi * R * nb + band;
    for (int c_pass = 0; c_pass < R; c_pass += G * CW) {
        const int c0 = c_pass + g * CW;
        int c_[CW];
#pragma unroll
        for (int j = 0; j < CW; ++j) c_[j] = 0;
        if (c0 < R) {
#pragma unroll 4
            for (int v = v_lo; v < v_hi; ++v) {
                const uint32_t pat = row_pattern<CW>(fl, (size_t)v * ld + c0);
#pragma unroll
                for (int j = 0; j < CW; ++j) c_[j] += (pat >> j) & 1u;
            }
        }
#pragma unroll
        for (int j = 0; j < CW; ++j) s_cnt[(g * CW + j) * S + s] = c_[j];
        __syncthreads();
        for (int k = threadIdx.x; k < G * CW; k += kThreads) {
            const int c = c_pass + k;
            if (c < R) {
                int t = 0;
                for (int q = 0; q < S; ++q) t += s_cnt[k * S + q];
                out[(size_t)c * nb] = t;
            }
        }
        __syncthreads();
    }
}

// One workgroup per CPI: the band counts become exclusive offsets in find() order (scan index
// c * nb + band), in place; count[cpi] = {total, 0}.
__global__ __launch_bounds__(kThreads) void band_scan_kernel(int R, int nb, int32_t* __restrict__ cnt,
                                                             int32_t* __restrict__ count) {
    __shared__ int s_wave[33];
    const int cpi = blockIdx.x;
    int32_t* base = cnt + (size_t)cpi * nb * R;
    const int64_t n = (int64_t)R * nb;
    const int64_t per = (n + kThreads - 1) / kThreads;
    const int64_t lo = min(n, (int64_t)threadIdx.x * per), hi = min(n, lo + per);
    int part = 0;
    for (int64_t k = lo; k < hi; ++k) part += base[k];   // contiguous chunk: loads issued together
    int total;
    int pre = block_scan(part, s_wave, &total);
    for (int64_t k = lo; k < hi; ++k) {
        const int x = base[k];
        base[k] = pre;
        pre += x;
    }
    if (threadIdx.x == 0) {
        count[cpi * 2 + 0] = total;
        count[cpi * 2 + 1] = 0;
    }
}

// The hits of band `band` into their slots: off[band][c] + the rows of column c above this
// thread's slice within the band.
template <int E, int CW>
__global__ __launch_bounds__(kThreads) void band_list_kernel(const uint8_t* __restrict__ flag, int V, int R, int G,
                                                             int64_t ld, int64_t cs, int nb, int Vb, int mtd0_num,
                                                             const int32_t* __restrict__ off, int64_t max_hits,
                                                             double* __restrict__ est, int32_t* __restrict__ count) {
    __shared__ int s_cnt[kThreads * CW];
    __shared__ int s_start[kThreads * CW];
    __shared__ int s_wave[33];
    __shared__ int s_bad;
    const int cpi = blockIdx.x / nb, band = blockIdx.x - cpi * nb;
    const uint8_t* fl = flag + cpi * cs;
    int64_t* hl = reinterpret_cast<int64_t*>(est) + (size_t)cpi * max_hits * 3;
    const int32_t* bo = off + (size_t)cpi * R * nb + band;   // column c at bo[c * nb]
    const int S = kThreads / G;
    const int g = threadIdx.x % G, s = threadIdx.x / G;
    const int b_lo = band * Vb, b_hi = min(V, b_lo + Vb);
    const int rows = (b_hi - b_lo + S - 1) / S;
    const int v_lo = min(b_hi, b_lo + s * rows), v_hi = min(b_hi, v_lo + rows);
    const int q = (rows + 63) / 64;
    if (threadIdx.x == 0) s_bad = 0;
    for (int c_pass = 0; c_pass < R; c_pass += G * CW) {
        const int c0 = c_pass + g * CW;
        int c_[CW];
#pragma unroll
        for (int j = 0; j < CW; ++j) c_[j] = 0;
        uint64_t rmask = 0;
        if (c0 < R) {
#pragma unroll 4
            for (int v = v_lo; v < v_hi; ++v) {
                const uint32_t pat = row_pattern<CW>(fl, (size_t)v * ld + c0);
#pragma unroll
                for (int j = 0; j < CW; ++j) c_[j] += (pat >> j) & 1u;
                rmask |= (uint64_t)(pat != 0) << ((v - v_lo) / q);
            }
        }
#pragma unroll
        for (int j = 0; j < CW; ++j) s_cnt[(g * CW + j) * S + s] = c_[j];
        __syncthreads();
        int run[CW], part = 0;
#pragma unroll
        for (int j = 0; j < CW; ++j) {
            run[j] = s_cnt[threadIdx.x * CW + j];
            part += run[j];
        }
        int total;
        int pre = block_scan(part, s_wave, &total);
#pragma unroll
        for (int j = 0; j < CW; ++j) {
            const int x = run[j];
            s_cnt[threadIdx.x * CW + j] = pre;   // within-band prefix P(column, slice)
            pre += x;
        }
        __syncthreads();
        // slot starts into a second array (P(column, 0) of other slices must stay readable)
#pragma unroll 1
        for (int j = 0; j < CW; ++j) {
            const int k = g * CW + j, c = c_pass + k;
            s_start[k * S + s] = c < R ? bo[(size_t)c * nb] + s_cnt[k * S + s] - s_cnt[k * S] : 0;
        }
        __syncthreads();
        while (rmask) {
            const int i = __builtin_ctzll(rmask);
            rmask &= rmask - 1;
            const int r_hi = min(v_hi, v_lo + (i + 1) * q);
            for (int v = v_lo + i * q; v < r_hi; ++v) {
                uint32_t pat = row_pattern<CW>(fl, (size_t)v * ld + c0);
                while (pat) {
                    const int j = __builtin_ctz(pat);
                    pat &= pat - 1;
                    const int c = c0 + j;
                    int* nx = &s_start[(g * CW + j) * S + s];
                    const int slot = *nx;
                    *nx = slot + 1;
                    if (slot < max_hits) {
                        hl[(size_t)slot * 3] = (int64_t)v * R + c;
                    } else {
                        int f0;
                        if (!fix_cells(c + 1, E, 1, R, R, &f0) ||
                            !fix_cells(v + 1, E, mtd0_num + 2, V - mtd0_num, V, &f0))
                            atomicAdd(&s_bad, 1);
                    }
                }
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0 && s_bad) atomicAdd(&count[cpi * 2 + 1], s_bad);
}

// One thread per listed hit (nb blocks per CPI): the cell index hits_kernel left in the first
// word of the slot is replaced by the slot's three estimates.
template <int E>
__global__ __launch_bounds__(256) void measure_kernel(const float* __restrict__ sum, const float* __restrict__ diff,
                                                      int V, int R, MeasureArgs a, const double* __restrict__ r_scale,
                                                      const double* __restrict__ v_scale, int64_t max_hits,
                                                      double* __restrict__ est, int32_t* __restrict__ cells,
                                                      int32_t* __restrict__ count, unsigned nb) {
    const int cpi = blockIdx.x / nb;
    const int64_t slot = (int64_t)(blockIdx.x - (unsigned)cpi * nb) * 256 + threadIdx.x;
    const int64_t n = count[cpi * 2];
    if (slot >= n || slot >= max_hits) return;
    const size_t plane = (size_t)a.cs;
    double* e = est + ((size_t)cpi * max_hits + slot) * 3;
    const int64_t idx = *reinterpret_cast<const int64_t*>(e);
    const int v = (int)(idx / R), c = (int)(idx - (int64_t)v * R);
    double e3[3];
    bool bad;
    measure_hit<E>(sum + cpi * plane, diff + cpi * plane, V, R, v, c, a, r_scale, v_scale, e3, &bad);
    e[0] = e3[0];
    e[1] = e3[1];
    e[2] = e3[2];
    if (cells) {
        cells[((size_t)cpi * max_hits + slot) * 2 + 0] = v;
        cells[((size_t)cpi * max_hits + slot) * 2 + 1] = c;
    }
    if (bad) atomicAdd(&count[cpi * 2 + 1], 1);
}

template <int E>
hipError_t launch_e(const float* sum, const float* diff, const uint8_t* flag, int V, int R, int batch,
                    const MeasureArgs& a, const double* r_scale, const double* v_scale, int64_t max_hits,
                    double* est, int32_t* cells, int32_t* count, int32_t* band_cnt, int nb, hipStream_t st) {
    const bool wide = R % 16 == 0 && R >= 16 * 16 && a.ld % 16 == 0 && a.cs % 16 == 0 && ((uintptr_t)flag & 15) == 0;
    // column groups per pass: a power of two covering the columns (16-byte groups: at least 16,
    // one 256-byte row segment per 16 lanes; bytes: at least 64), at most 1024
    int G = wide ? 16 : 64;
    const int groups = wide ? R / 16 : R;
    while (G < groups && G < kThreads) G <<= 1;
    if (nb > 1) {   // banded: nb workgroups per CPI
        const int Vb = (V + nb - 1) / nb;
        const unsigned grid = (unsigned)((int64_t)batch * nb);
        if (wide)
            hipLaunchKernelGGL((band_count_kernel<16>), dim3(grid), dim3(kThreads), 0, st, flag, V, R, G, a.ld, a.cs,
                               nb, Vb, band_cnt);
        else
            hipLaunchKernelGGL((band_count_kernel<1>), dim3(grid), dim3(kThreads), 0, st, flag, V, R, G, a.ld, a.cs,
                               nb, Vb, band_cnt);
        hipLaunchKernelGGL(band_scan_kernel, dim3(batch), dim3(kThreads), 0, st, R, nb, band_cnt, count);
        if (wide)
            hipLaunchKernelGGL((band_list_kernel<E, 16>), dim3(grid), dim3(kThreads), 0, st, flag, V, R, G, a.ld,
                               a.cs, nb, Vb, a.mtd0_num, band_cnt, max_hits, est, count);
        else
            hipLaunchKernelGGL((band_list_kernel<E, 1>), dim3(grid), dim3(kThreads), 0, st, flag, V, R, G, a.ld,
                               a.cs, nb, Vb, a.mtd0_num, band_cnt, max_hits, est, count);
    } else if (wide) {
        hipLaunchKernelGGL((hits_kernel<E, 16>), dim3(batch), dim3(kThreads), 0, st, flag, V, R, G, a.ld, a.cs, a.mtd0_num,
                           max_hits, est, count);
    } else {
        hipLaunchKernelGGL((hits_kernel<E, 1>), dim3(batch), dim3(kThreads), 0, st, flag, V, R, G, a.ld, a.cs, a.mtd0_num,
                           max_hits, est, count);
    }
    hipError_t err = hipGetLastError();
    if (err != hipSuccess || max_hits == 0) return err;
    // slots past a CPI's hit count exit at once; the grid covers max_hits (capped by V*R)
    const int64_t cap = max_hits < (int64_t)V * R ? max_hits : (int64_t)V * R;
    const int64_t nbk = (cap + 255) / 256, blocks = nbk * batch;   // blocks per CPI, total (1-D grid)
    if (blocks > 0x7fffffff) return hipErrorInvalidConfiguration;
    hipLaunchKernelGGL((measure_kernel<E>), dim3((unsigned)blocks), dim3(256), 0, st, sum, diff, V, R, a, r_scale,
                       v_scale, max_hits, est, cells, count, (unsigned)nbk);
    return hipGetLastError();
}

}  // namespace

// Dev-only build (-DRSP_DEV_MEASURE_BANDS=N > 1, tools/build_variant.sh): N bands per CPI for
// batches below the CU count.
// Measured slower than one workgroup per CPI at every batch tried (2048 x 512, ~1044 hits:
// batch 1 113 vs 64 us, batch 8 84 vs 65 us, batch 64 100 vs 79 us per call): its three
// launches each cost more than the single workgroup's whole flag scan (band_scan alone 50 us
// of dependent loads in one workgroup).  Bit-exact against the oracle when enabled.
int measure_bands(int V, int batch) {
#ifdef RSP_DEV_MEASURE_BANDS
    const int want = RSP_DEV_MEASURE_BANDS;
#else
    const int want = 1;
#endif
    if (want <= 1 || batch >= 128) return 1;
    const int max_nb = (V + 31) / 32;                      // bands of at least 32 rows
    return want < max_nb ? want : max_nb;
}

hipError_t launch_measure(const float* sum, const float* diff, const uint8_t* flag, int V, int R, int batch,
                          const MeasureArgs& a, const double* r_scale, const double* v_scale, int64_t max_hits,
                          double* est, int32_t* cells, int32_t* count, int32_t* band_cnt, int nb, hipStream_t st) {
    if (batch <= 0) return hipSuccess;
    switch (a.extra_dots) {
        case 1: return launch_e<1>(sum, diff, flag, V, R, batch, a, r_scale, v_scale, max_hits, est, cells, count, band_cnt, nb, st);
        case 2: return launch_e<2>(sum, diff, flag, V, R, batch, a, r_scale, v_scale, max_hits, est, cells, count, band_cnt, nb, st);
        case 3: return launch_e<3>(sum, diff, flag, V, R, batch, a, r_scale, v_scale, max_hits, est, cells, count, band_cnt, nb, st);
        case 4: return launch_e<4>(sum, diff, flag, V, R, batch, a, r_scale, v_scale, max_hits, est, cells, count, band_cnt, nb, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace rsp
