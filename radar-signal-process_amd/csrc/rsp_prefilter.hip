// rsp_prefilter.hip -- the reference's echo pre-filters for gfx950:
//   * iSTC  (MTD/fun_iSTC.m:12-15): echo(i,:) .* 10.^(stc/20), a per-range-bin gain;
//   * MTI   (MTD/fun_Process_MTI.m:20-22): out(m,:) = x(m+lag,:) - x(m,:) for m <= P-lag
//           (lag 30 in the reference), rows past P-lag stay zero (:9).
// Both are elementwise over the [batch][P][R] complex64 echo (row = pulse, contiguous range):
// one thread per 2 complex samples (16-byte loads and stores), the gain read once per thread
// pair, so the kernel is a pure HBM stream: 8 B read + 8 B written per sample.  MTI runs as
// chains (mti_chain_kernel): a thread walks the rows r, r+lag, ... of one sample pair, so each
// sample is still loaded once.
// The gains are computed on the host in fp64 (rsp/prefilter.py); the products are fp32.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/rsp.h"
#include "rsp_internal.h"

namespace rsp {

namespace {

__device__ __forceinline__ float4 cmul_gain(float4 x, float g0, float g1) {
    return make_float4(x.x * g0, x.y * g0, x.z * g1, x.w * g1);
}

// R2 = R / 2 sample pairs per row; `pairs` = batch * P * R2 in total.
template <bool GAIN, bool MTI>
__global__ __launch_bounds__(256) void prefilter_kernel(const float4* __restrict__ in, float4* __restrict__ out,
                                                        const float2* __restrict__ gain, int P, int R2, int lag,
                                                        int64_t pairs) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < pairs; i += stride) {
        const int64_t row = i / R2;
        const int c = (int)(i - row * R2);
        const int m = (int)(row % P);
        float4 y;
        if constexpr (MTI) {
            if (m + lag < P) {
                const float4 a = in[i + (int64_t)lag * R2], b = in[i];
                y = make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w);
            } else {
                y = make_float4(0.f, 0.f, 0.f, 0.f);
            }
        } else {
            y = in[i];
        }
        if constexpr (GAIN) {
            const float2 g = gain[c];
            y = cmul_gain(y, g.x, g.y);
        }
        out[i] = y;
    }
}

// MTI as chains: thread (CPI b, phase r < lag, sample pair c) walks rows r, r+lag, r+2*lag, ...
// keeping the previous row's value, so every input sample is loaded exactly once (the
// row-parallel form fetches x(m+lag) a second time, from another XCD's L2 or from HBM).
template <bool GAIN>
__global__ __launch_bounds__(256) void mti_chain_kernel(const float4* __restrict__ in, float4* __restrict__ out,
                                                        const float2* __restrict__ gain, int P, int R2, int lag,
                                                        int chains, int64_t items) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < items; i += stride) {
        const int64_t rest = i / R2;
        const int c = (int)(i - rest * R2);
        const int64_t b = rest / chains;
        const int r = (int)(rest - b * chains);
        float g0 = 1.f, g1 = 1.f;
        if constexpr (GAIN) {
            const float2 g = gain[c];
            g0 = g.x;
            g1 = g.y;
        }
        const int64_t base = b * P * (int64_t)R2 + c;
        const int64_t step = (int64_t)lag * R2;
        int m = r;
        float4 prev = make_float4(0.f, 0.f, 0.f, 0.f);
        if (m + lag < P) prev = in[base + (int64_t)m * R2];
        for (; m + lag < P; m += lag) {
            const float4 next = in[base + (int64_t)m * R2 + step];
            float4 y = make_float4(next.x - prev.x, next.y - prev.y, next.z - prev.z, next.w - prev.w);
            if constexpr (GAIN) y = cmul_gain(y, g0, g1);
            out[base + (int64_t)m * R2] = y;
            prev = next;
        }
        for (; m < P; m += lag) out[base + (int64_t)m * R2] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

template <bool GAIN>
hipError_t launch_chain(const float4* in, float4* out, const float2* gain, int P, int R2, int lag, int64_t batch,
                        hipStream_t st) {
    const int chains = lag < P ? lag : P;
    const int64_t items = batch * chains * (int64_t)R2;
    int64_t blocks = (items + 255) / 256;
    if (blocks > 256 * 64) blocks = 256 * 64;
    hipLaunchKernelGGL((mti_chain_kernel<GAIN>), dim3((unsigned)blocks), dim3(256), 0, st, in, out, gain, P, R2, lag,
                       chains, items);
    return hipGetLastError();
}

template <bool GAIN, bool MTI>
hipError_t launch_t(const float4* in, float4* out, const float2* gain, int P, int R2, int lag, int64_t pairs,
                    hipStream_t st) {
    int64_t blocks = (pairs + 255) / 256;
    if (blocks > 256 * 64) blocks = 256 * 64;   // grid-stride beyond 64 workgroups per CU
    hipLaunchKernelGGL((prefilter_kernel<GAIN, MTI>), dim3((unsigned)blocks), dim3(256), 0, st, in, out, gain, P, R2,
                       lag, pairs);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_prefilter(const float2* in, float2* out, const float* gain, int P, int R, int64_t batch, int lag,
                            hipStream_t st) {
    const int64_t pairs = batch * P * (int64_t)(R / 2);
    if (pairs == 0) return hipSuccess;
    const float4* i4 = reinterpret_cast<const float4*>(in);
    float4* o4 = reinterpret_cast<float4*>(out);
    const float2* g2 = reinterpret_cast<const float2*>(gain);
#ifdef RSP_DEV_MTI_ROWWISE   // dev-only build (tools/build_variant.sh): the row-parallel form, measured slower
    constexpr bool rowwise = true;
#else
    constexpr bool rowwise = false;
#endif
    if (lag > 0 && !rowwise)
        return gain ? launch_chain<true>(i4, o4, g2, P, R / 2, lag, batch, st)
                    : launch_chain<false>(i4, o4, g2, P, R / 2, lag, batch, st);
    if (gain && lag > 0) return launch_t<true, true>(i4, o4, g2, P, R / 2, lag, pairs, st);
    if (gain) return launch_t<true, false>(i4, o4, g2, P, R / 2, lag, pairs, st);
    if (lag > 0) return launch_t<false, true>(i4, o4, g2, P, R / 2, lag, pairs, st);
    return launch_t<false, false>(i4, o4, g2, P, R / 2, lag, pairs, st);
}

}  // namespace rsp
