// rsp_ingest.hip -- raw-data ingest for gfx950: the PRT record codec of FrameDataRead_xzr.m
// (64-B head of uint32 fields, 128-B realtime block, int16 I/Q DDC payload padded to 64 B,
// 64-B tail) and the DBF beamforming product sig_data_C * DBF_coeffs_data_C.' of every
// sample (FrameDataRead_xzr.m:149-158), straight into the beam-major echo layout
// [beam][prt][sample] that the PC -> MTD chain reads.
//
// Two launches per frame, both on the caller's stream:
//   ingest_check_kernel  one workgroup, a thread per PRT: validates its head against the
//                        frame shape and the byte count, writes a status code, and reduces
//                        the first PRT the frame cannot get past into status[prt_num];
//   ingest_ddc_kernel    one thread per (PRT, sample): 16-byte loads of the sample's
//                        channel I/Q words, fp32 DBF with the coefficients read as scalars
//                        (wave-uniform), one coalesced 8-byte store per beam; rows at or
//                        after the stop PRT are written as zeros (the reference returns
//                        with the rest of sig_data_DBF_allprts still zero, :43,63-66).
// The record layout is uniform within a frame (every DDC PRT has the same size); a head
// that disagrees is a status code, as the reference's size check makes it a failed frame.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rsp.h"
#include "rsp_buf.h"
#include "rsp_internal.h"

namespace rsp {

// Head words (uint32, little-endian; FrameDataRead_xzr.m:74-86): [2] PRT number (low 16) and
// frequency number, [3] channel count (low 8), [4] servo angle in 0.1 deg (low 16), [6] samples
// per PRT, [7] data type (low 8) | PRT count (bits 8-23) | radar type (bits 24-31).
constexpr int kHwChannels = 3, kHwServo = 4, kHwPulseDataNum = 6, kHwType = 7;

// One workgroup checks every PRT of the frame (a frame has a few hundred) and reduces the
// stop row in LDS, so status[] needs no initialisation pass.
__global__ __launch_bounds__(1024) void ingest_check_kernel(const uint8_t* __restrict__ stream, int64_t nbytes,
                                                             IngestArgs a, uint16_t* __restrict__ servo,
                                                             int32_t* __restrict__ status) {
    __shared__ int s_stop;
    if (threadIdx.x == 0) s_stop = a.prt_num;
    __syncthreads();
    for (int p = threadIdx.x; p < a.prt_num; p += blockDim.x) {
        const int64_t base = (int64_t)p * a.rec_bytes;
        int32_t st = RSP_PRT_OK;
        int stop = a.prt_num;   // first row this PRT keeps from being decoded
        if (base + a.bytes_head > nbytes) {
            st = RSP_PRT_TRUNCATED;                      // :62-67
            stop = p;
        } else {
            const uint32_t* h = reinterpret_cast<const uint32_t*>(stream + base);
            const uint32_t pdn = h[kHwPulseDataNum];
            const uint32_t ch = h[kHwChannels] & 0xffu;
            const uint32_t type = h[kHwType] & 0xffu;
            if ((int32_t)pdn <= 0) {
                st = RSP_PRT_BAD_COUNT;                  // :90-94
                stop = p;
            } else if (type != 1u) {
                st = RSP_PRT_UNSUPPORTED_TYPE;           // ADC / DBF payloads: not built
                stop = p;
            } else if ((int)ch != a.channel_num || (int)pdn != a.point_prt) {
                st = RSP_PRT_BAD_SHAPE;                  // :171-176 (and the DBF product's inner dimension)
                stop = p;
            } else if (base + a.rec_bytes - a.bytes_tail > nbytes) {
                st = RSP_PRT_TRUNCATED;                  // realtime block or payload cut (:97-127)
                stop = p;
            } else if (base + a.rec_bytes > nbytes) {
                st = RSP_PRT_TAIL_TRUNCATED;             // stored, then the tail read fails (:179-189)
                stop = p + 1;
            }
            if (servo) servo[p] = (uint16_t)(h[kHwServo] & 0xffffu);   // zeroed below for rows past the stop
        }
        status[p] = st;
        if (stop < a.prt_num) atomicMin(&s_stop, stop);
    }
    __syncthreads();
    if (threadIdx.x == 0) status[a.prt_num] = s_stop;
}

// out[b * beam_stride + p * point + s] = sum_c (I_c + j Q_c) * C[b][c], fp32 in channel order.
// CH > 0 / NB > 0: compile-time channel and beam counts (the v2 capture's 16 and 13): every
// beam's sum is formed before the first store, so the coefficients' scalar loads never have
// to wait for the stores (a scalar load after a vector store to memory that may alias it
// costs a vmcnt(0) drain per beam otherwise).
template <int CH, int NB>
__global__ __launch_bounds__(256) void ingest_ddc_kernel(const uint8_t* __restrict__ stream, IngestArgs a,
                                                          const float2* __restrict__ dbf, float2* __restrict__ out,
                                                          uint16_t* __restrict__ servo,
                                                          const int32_t* __restrict__ status) {
    const int p = blockIdx.y;
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    const int stop = status[a.prt_num];
    const int ch = CH > 0 ? CH : a.channel_num;
    if (servo && p >= stop && blockIdx.x == 0 && threadIdx.x == 0) servo[p] = 0;
    if (s >= a.point_prt) return;
    const size_t o = (size_t)p * a.point_prt + s;
    if (p >= stop) {
        for (int b = 0; b < a.beam_num; ++b) out[(size_t)b * a.beam_stride + o] = make_float2(0.f, 0.f);
        return;
    }
    // the PRT's payload as a buffer resource: the sample's channel words at s * ch * 4
    const uint8_t* pay = stream + (int64_t)p * a.rec_bytes + a.bytes_head + a.bytes_realtime;
    const auto pr = buf_rsrc(pay, (uint32_t)a.point_prt * (uint32_t)ch * 4u);
    if constexpr (CH > 0 && NB > 0) {
        static_assert(CH % 4 == 0, "16-byte loads of 4 channels");
        typedef int v4i __attribute__((ext_vector_type(4)));
        float2 x[CH];
#pragma unroll
        for (int q = 0; q < CH / 4; ++q) {
            const v4i w = __builtin_bit_cast(
                v4i, __builtin_amdgcn_raw_buffer_load_b128(pr, (uint32_t)s * (CH * 4u), (uint32_t)q * 16u, 0));
#pragma unroll
            for (int k = 0; k < 4; ++k)   // low half I, high half Q (:150-156)
                x[4 * q + k] = make_float2((float)(int16_t)(w[k] & 0xffff), (float)(int16_t)((uint32_t)w[k] >> 16));
        }
        float2 acc[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            acc[b] = make_float2(0.f, 0.f);
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                const float2 w = dbf[b * CH + c];   // wave-uniform: scalar loads
                acc[b].x = fmaf(x[c].x, w.x, fmaf(-x[c].y, w.y, acc[b].x));
                acc[b].y = fmaf(x[c].x, w.y, fmaf(x[c].y, w.x, acc[b].y));
            }
        }
#pragma unroll
        for (int b = 0; b < NB; ++b) out[(size_t)b * a.beam_stride + o] = acc[b];
    } else {
        for (int b = 0; b < a.beam_num; ++b) {
            const float2* cb = dbf + (size_t)b * ch;
            float2 acc = make_float2(0.f, 0.f);
            for (int c = 0; c < ch; ++c) {
                const uint32_t w = __builtin_amdgcn_raw_buffer_load_b32(pr, (uint32_t)(s * ch + c) * 4u, 0u, 0);
                const float xi = (float)(int16_t)(w & 0xffff), xq = (float)(int16_t)(w >> 16);
                const float2 cw = cb[c];
                acc.x = fmaf(xi, cw.x, fmaf(-xq, cw.y, acc.x));
                acc.y = fmaf(xi, cw.y, fmaf(xq, cw.x, acc.y));
            }
            out[(size_t)b * a.beam_stride + o] = acc;
        }
    }
}

hipError_t launch_ingest_ddc(const uint8_t* stream, int64_t nbytes, const IngestArgs& a, const float2* dbf,
                             float2* out, uint16_t* servo, int32_t* status, hipStream_t s) {
    if (a.prt_num <= 0) return hipSuccess;
    hipLaunchKernelGGL(ingest_check_kernel, dim3(1), dim3(1024), 0, s, stream, nbytes, a, servo, status);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const dim3 grid((unsigned)((a.point_prt + 255) / 256), (unsigned)a.prt_num);
    if (a.channel_num == 16 && a.beam_num == 13)   // the v2 capture (bin_to_mat_xzr.m:39-40)
        hipLaunchKernelGGL((ingest_ddc_kernel<16, 13>), grid, dim3(256), 0, s, stream, a, dbf, out, servo, status);
    else
        hipLaunchKernelGGL((ingest_ddc_kernel<0, 0>), grid, dim3(256), 0, s, stream, a, dbf, out, servo, status);
    return hipGetLastError();
}

}  // namespace rsp
