// rsp_ingest.hip -- raw-data ingest for gfx950: the PRT record codec of FrameDataRead_xzr.m
// (64-B head of uint32 fields, 128-B realtime block, payload padded to 64 B, 64-B tail) and
// the payload decode of every data type straight into the beam-major echo layout
// [beam][prt][sample] that the PC -> MTD chain reads:
//   DDC (type 1)   int16 I/Q per channel, then the DBF product sig_data_C * DBF_coeffs_data_C.'
//                  (FrameDataRead_xzr.m:149-158);
//   ADC (type 0)   int16 per channel, the (samples x channels) matrix itself (:144-147), which
//                  passes the size check only with channel_num == beam_num;
//   DBF (type 2)   the 24-bit branch (:130-135,162-164) as MATLAB evaluates it: data_temp is
//                  uint8, so b0 + b1*2^8 + b2*2^16 saturates (255 once b1 or b2 is non-zero,
//                  else b0) and the > 2^23 sign fix never fires; value pairs form the I/Q
//                  columns.  (The reference marks this branch unfinished; its results are
//                  reproduced as it computes them.)
//   types 3..255   payload sized as DBF (:110-112) and read, no switch case (:160-165): the row
//                  is zeros(point_PRT, beam_num), which passes the :171 size check.
//
// Two launches per frame, both on the caller's stream:
//   ingest_check_kernel  one workgroup, a thread per PRT: locates its record, validates the
//                        head against the frame shape and the byte count, writes a status
//                        code, and reduces the first PRT the frame cannot get past into
//                        status[prt_num].  Records are located speculatively at p * (size of
//                        PRT 0's record); the first PRT whose head implies another size ends the
//                        speculation and one thread walks the heads from there (mixed frames);
//   ingest_decode_kernel one thread per (PRT, sample), the PRT's type a block-uniform branch;
//                        DDC: 16-byte loads of the sample's channel I/Q words, fp32 DBF with the
//                        coefficients read as scalars (wave-uniform), one coalesced 8-byte store
//                        per beam; rows at or after the stop PRT are written as zeros (the
//                        reference returns with the rest of sig_data_DBF_allprts still zero,
//                        :43,63-66).
// rsp_ingest_ddc_dev keeps the DDC-only contract: records sized by the params, other types a
// status code.
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

struct RecHead {
    uint32_t pdn, ch, type, servo;
};
__device__ __forceinline__ RecHead read_head(const uint8_t* stream, int64_t base) {
    const uint32_t* h = reinterpret_cast<const uint32_t*>(stream + base);
    return RecHead{h[kHwPulseDataNum], h[kHwChannels] & 0xffu, h[kHwType] & 0xffu, h[kHwServo] & 0xffffu};
}
__device__ __forceinline__ int64_t record_bytes(const IngestArgs& a, const RecHead& h) {
    return (int64_t)a.bytes_head + a.bytes_realtime + ingest_payload_bytes(h.type, h.pdn, h.ch) + a.bytes_tail;
}

// Status of the record at `base` (the reference's early returns in its read order: head,
// pulse_data_num, realtime block, payload, size check, tail) and the first row it keeps from
// being decoded (p, p + 1 for a cut tail, or prt_num).
__device__ __forceinline__ int32_t check_record(const uint8_t* stream, int64_t nbytes, const IngestArgs& a, int p,
                                                int64_t base, int* stop, uint16_t* servo) {
    *stop = p;
    if (base + a.bytes_head > nbytes) return RSP_PRT_TRUNCATED;               // :62-67
    const RecHead h = read_head(stream, base);
    if (servo) servo[p] = (uint16_t)h.servo;   // zeroed by the decode kernel for rows past the stop
    if (a.ddc_only) {
        if (h.pdn == 0u) return RSP_PRT_BAD_COUNT;
        if (h.type != 1u) return RSP_PRT_UNSUPPORTED_TYPE;
        if ((int)h.ch != a.channel_num || (int)h.pdn != a.point_prt) return RSP_PRT_BAD_SHAPE;
        if (base + a.rec_bytes - a.bytes_tail > nbytes) return RSP_PRT_TRUNCATED;
        if (base + a.rec_bytes > nbytes) {
            *stop = p + 1;
            return RSP_PRT_TAIL_TRUNCATED;
        }
        *stop = a.prt_num;
        return RSP_PRT_OK;
    }
    if (h.pdn == 0u) return RSP_PRT_BAD_COUNT;                               // :90-94 (uint32: only 0)
    const int64_t rec = record_bytes(a, h);
    if (base + rec - a.bytes_tail > nbytes) return RSP_PRT_TRUNCATED;        // :97-127
    bool shape;                                                             // :171-176
    if (h.type == 1u) shape = (int)h.ch == a.channel_num && (int)h.pdn == a.point_prt;   // (and :158's inner dimension)
    else if (h.type == 0u) shape = (int)h.ch == a.beam_num && (int)h.pdn == a.point_prt;
    else if (h.type == 2u) shape = dbf24_values((int)h.ch) == 2 * a.beam_num && (int)h.pdn == a.point_prt;
    else shape = true;   // types 3..255: no switch case matches, the zeros(point_PRT, beam_num) row passes
    if (!shape) return RSP_PRT_BAD_SHAPE;
    if (base + rec > nbytes) {                                              // stored, then :184-189
        *stop = p + 1;
        return RSP_PRT_TAIL_TRUNCATED;
    }
    *stop = a.prt_num;
    return RSP_PRT_OK;
}

// One workgroup checks every PRT of the frame (a frame has a few hundred) and reduces the
// stop row in LDS, so status[] needs no initialisation pass.
__global__ __launch_bounds__(1024) void ingest_check_kernel(const uint8_t* __restrict__ stream, int64_t nbytes,
                                                             IngestArgs a, uint16_t* __restrict__ servo,
                                                             int32_t* __restrict__ status) {
    __shared__ int s_stop, s_split;
    __shared__ int64_t s_rec0;
    if (threadIdx.x == 0) {
        s_stop = a.prt_num;
        s_split = a.prt_num;
        s_rec0 = a.rec_bytes;
        if (!a.ddc_only && a.bytes_head <= nbytes) {
            const RecHead h = read_head(stream, 0);
            if (h.pdn != 0u) s_rec0 = record_bytes(a, h);
        }
    }
    __syncthreads();
    const int64_t rec0 = s_rec0;
    if (!a.ddc_only) {
        // the speculation holds up to the first readable head whose record size is not rec0
        for (int p = threadIdx.x; p < a.prt_num; p += blockDim.x) {
            const int64_t base = (int64_t)p * rec0;
            if (base + a.bytes_head > nbytes) continue;
            const RecHead h = read_head(stream, base);
            if (h.pdn == 0u || record_bytes(a, h) != rec0) atomicMin(&s_split, p);
        }
        __syncthreads();
        if (threadIdx.x == 0 && s_split < a.prt_num) {   // mixed frame: walk the heads from the split
            int64_t off = (int64_t)s_split * rec0;
            for (int q = s_split; q < a.prt_num; ++q) {
                a.offs[q] = off;
                if (off + a.bytes_head > nbytes) continue;   // (rows from here on are not decoded)
                const RecHead h = read_head(stream, off);
                if (h.pdn == 0u) {
                    off = nbytes;
                    continue;
                }
                off += record_bytes(a, h);
            }
        }
        __syncthreads();   // (also orders thread 0's offsets before the other threads read them)
    }
    const int split = s_split;
    for (int p = threadIdx.x; p < a.prt_num; p += blockDim.x) {
        const int64_t base = p < split ? (int64_t)p * rec0 : a.offs[p];
        int stop;
        const int32_t st = check_record(stream, nbytes, a, p, base, &stop, servo);
        status[p] = st;
        a.offs[p] = base;
        if (base + a.bytes_head <= nbytes) {   // type | channel count << 8 (decoded rows only)
            const RecHead h = read_head(stream, base);
            a.types[p] = (int32_t)(h.type | (h.ch << 8));
        }
        if (stop < a.prt_num) atomicMin(&s_stop, stop);
    }
    __syncthreads();
    if (threadIdx.x == 0) status[a.prt_num] = s_stop;
}

// out[b * beam_stride + p * point + s]: DDC sum_c (I_c + j Q_c) * C[b][c] in fp32, channel order;
// ADC (x_b, 0); DBF the saturated value pair (v_2b, v_2b+1).
// CH > 0 / NB > 0: compile-time channel and beam counts of the DDC path (the v2 capture's 16 and
// 13): every beam's sum is formed before the first store, so the coefficients' scalar loads
// never have to wait for the stores (a scalar load after a vector store to memory that may
// alias it costs a vmcnt(0) drain per beam otherwise).
template <int CH, int NB>
__global__ __launch_bounds__(256) void ingest_decode_kernel(const uint8_t* __restrict__ stream, IngestArgs a,
                                                             const float2* __restrict__ dbf, float2* __restrict__ out,
                                                             uint16_t* __restrict__ servo,
                                                             const int32_t* __restrict__ status) {
    const int p = blockIdx.y;
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    // generic shapes: the DBF matrix staged in LDS once per block (the host passes its size as
    // dynamic LDS when it fits, else 0): per beam the channel sums then read their coefficients
    // as LDS broadcasts, where scalar loads behind each beam's vector stores cost a vmcnt(0) drain
    extern __shared__ float2 s_dbf[];
    constexpr int kChMax = 32;   // channels a thread holds in registers on that path
    const bool staged = CH == 0 && a.dbf_lds != 0;
    if (staged) {
        for (int i = threadIdx.x; i < a.beam_num * a.channel_num; i += blockDim.x) s_dbf[i] = dbf[i];
        __syncthreads();
    }
    const int stop = status[a.prt_num];
    if (servo && p >= stop && blockIdx.x == 0 && threadIdx.x == 0) servo[p] = 0;
    if (s >= a.point_prt) return;
    const size_t o = (size_t)p * a.point_prt + s;
    if (p >= stop) {
        for (int b = 0; b < a.beam_num; ++b) out[(size_t)b * a.beam_stride + o] = make_float2(0.f, 0.f);
        return;
    }
    const int type = a.types[p] & 0xff;
    const uint8_t* pay = stream + a.offs[p] + a.bytes_head + a.bytes_realtime;
    if (type == 0) {   // ADC: channel b is beam b (channel_num == beam_num, checked)
        const int ch = a.beam_num;
        const auto pr = buf_rsrc(pay, (uint32_t)a.point_prt * (uint32_t)ch * 2u);
        for (int b = 0; b < a.beam_num; ++b) {
            const uint32_t w = __builtin_amdgcn_raw_buffer_load_b16(pr, (uint32_t)(s * ch + b) * 2u, 0u, 0);
            out[(size_t)b * a.beam_stride + o] = make_float2((float)(int16_t)w, 0.f);
        }
        return;
    }
    if (type > 2) {   // types 3..255 (:160-165 has no case): the row stays zeros(point_PRT, beam_num)
        for (int b = 0; b < a.beam_num; ++b) out[(size_t)b * a.beam_stride + o] = make_float2(0.f, 0.f);
        return;
    }
    if (type == 2) {   // 24-bit DBF branch as MATLAB's uint8 arithmetic evaluates it
        const uint32_t L = (uint32_t)dbf24_row_bytes(a.types[p] >> 8);   // the PRT's own channel count
        const auto pr = buf_rsrc(pay, (uint32_t)a.point_prt * L);
        const uint32_t row = (uint32_t)s * L;
        for (int b = 0; b < a.beam_num; ++b) {
            float v[2];
#pragma unroll
            for (int k = 0; k < 2; ++k) {   // value j = 2b + k: bytes 3j, 3j + 1, 3j + 2 of the sample row
                const uint32_t j3 = 3u * (uint32_t)(2 * b + k);
                const uint32_t b0 = __builtin_amdgcn_raw_buffer_load_b8(pr, row + j3, 0u, 0);
                const uint32_t b1 = __builtin_amdgcn_raw_buffer_load_b8(pr, row + j3 + 1u, 0u, 0);
                const uint32_t b2 = __builtin_amdgcn_raw_buffer_load_b8(pr, row + j3 + 2u, 0u, 0);
                v[k] = (float)((b1 | b2) ? 255u : b0);   // uint8 saturation of b0 + b1*2^8 + b2*2^16
            }
            out[(size_t)b * a.beam_stride + o] = make_float2(v[0], v[1]);
        }
        return;
    }
    const int ch = CH > 0 ? CH : a.channel_num;
    // the PRT's payload as a buffer resource: the sample's channel words at s * ch * 4
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
    } else if (staged && ch <= kChMax) {   // the sample's channels loaded once, in registers
        float2 x[kChMax];
#pragma unroll
        for (int c = 0; c < kChMax; ++c) {
            if (c < ch) {   // (uniform)
                const uint32_t w = __builtin_amdgcn_raw_buffer_load_b32(pr, (uint32_t)(s * ch + c) * 4u, 0u, 0);
                x[c] = make_float2((float)(int16_t)(w & 0xffff), (float)(int16_t)(w >> 16));
            }
        }
        for (int b = 0; b < a.beam_num; ++b) {
            const float2* cb = s_dbf + b * ch;
            float2 acc = make_float2(0.f, 0.f);
#pragma unroll
            for (int c = 0; c < kChMax; ++c) {
                if (c < ch) {   // (uniform; the same sums in the same order as below)
                    const float2 cw = cb[c];
                    acc.x = fmaf(x[c].x, cw.x, fmaf(-x[c].y, cw.y, acc.x));
                    acc.y = fmaf(x[c].x, cw.y, fmaf(x[c].y, cw.x, acc.y));
                }
            }
            out[(size_t)b * a.beam_stride + o] = acc;
        }
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

hipError_t launch_ingest(const uint8_t* stream, int64_t nbytes, const IngestArgs& a, const float2* dbf,
                         float2* out, uint16_t* servo, int32_t* status, hipStream_t s) {
    if (a.prt_num <= 0) return hipSuccess;
    hipLaunchKernelGGL(ingest_check_kernel, dim3(1), dim3(1024), 0, s, stream, nbytes, a, servo, status);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const dim3 grid((unsigned)((a.point_prt + 255) / 256), (unsigned)a.prt_num);
    if (a.channel_num == 16 && a.beam_num == 13)   // the v2 capture (bin_to_mat_xzr.m:39-40)
        hipLaunchKernelGGL((ingest_decode_kernel<16, 13>), grid, dim3(256), 0, s, stream, a, dbf, out, servo, status);
    else {
        IngestArgs g = a;
        const size_t lds = (size_t)a.beam_num * (size_t)a.channel_num * sizeof(float2);
        g.dbf_lds = lds <= 32768 ? 1 : 0;   // (within the default dynamic-LDS limit)
        hipLaunchKernelGGL((ingest_decode_kernel<0, 0>), grid, dim3(256), g.dbf_lds ? lds : 0, s, stream, g, dbf, out,
                           servo, status);
    }
    return hipGetLastError();
}

}  // namespace rsp
