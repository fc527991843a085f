// Raw buffer access for gfx950 (device code only).
//
// A buffer resource (V#) covers one CPI plane; lanes address it with a 32-bit per-lane
// voffset plus a wave-uniform soffset, so strided slow-time / Doppler-row accesses put
// their row stride in an SGPR and spend no VALU on 64-bit address arithmetic.  The
// hardware range check (offset >= num_records) makes loads return 0 and drops stores,
// which replaces per-element `if (in range)` branches: a lane that must not touch memory
// uses kOob as its voffset.
#pragma once
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rsp {

constexpr int kBufWord3 = 0x00020000;    // gfx9 resource word 3 (raw, 32-bit data format)
constexpr uint32_t kOob = 0x80000000u;   // voffset beyond any plane (planes are < 2 GiB)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, kBufWord3);
}

__device__ __forceinline__ float2 buf_ld_f2(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}
__device__ __forceinline__ float buf_ld_f(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
__device__ __forceinline__ void buf_st_f2(float2 v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    typedef int v2i __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2i, v), r, voff, soff, 0);
}
__device__ __forceinline__ void buf_st_f(float v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, voff, soff, 0);
}
__device__ __forceinline__ void buf_st_u8(uint8_t v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_buffer_store_b8(v, r, voff, soff, 0);
}

// Cache policy of the streamed-once planes (echo input, RDM output): the default.  Marking
// them non-temporal (aux bit 1, `nt`) so they would not evict the PC scratch was measured
// slower (the range stage re-reads RDM neighbourhoods, and PC gains nothing).
constexpr int kStreamAux = 0;

// one complex element of an input plane (complex fp32, or fp16 I/Q widened on load).  The fp16
// echo (config c5: 512 x 16384, a 67 MB PC scratch per CPI and pipeline, near the 256 MB
// Infinity Cache with two pipelines) is loaded non-temporal (aux bit 1, `nt`): read once, it
// then evicts less of the scratch (c5 +2 %).  The same hint on the fp32 echo was neutral at c3
// and cost c4 3 %, and on the MTD's scratch loads cost c3 2 % and c5 2 %.
constexpr int kEchoF16Aux = 2;
__device__ __forceinline__ float2 buf_ld_c(const float2*, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, kStreamAux));
}
__device__ __forceinline__ float2 buf_ld_c(const __half2*, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __half22float2(__builtin_bit_cast(__half2, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, kEchoF16Aux)));
}
// streamed-once store (RDM)
__device__ __forceinline__ void buf_st_f_stream(float v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, voff, soff, kStreamAux);
}

// ---------------------------------------------------------------- in-launch hand-offs
// The fused chain (chain_kernel) hands PC rows, RDM tiles and hit lists between workgroups
// inside one launch.  Per-XCD L2s are not coherent, so every handed-off byte is stored
// write-through (`sc1`, cache-policy aux 16) and every load of it is an `sc1` load (L1
// bypassed, no acquire fence), with one agent-scope counter add per producing workgroup
// after all its waves drained vmcnt (cdna_hip_programming.md Guideline 16, valid-form row 1).
// Aux template argument: 0 = default policy, kSc1 = write-through / L1-bypass.
constexpr int kSc1 = 16;   // aux bits of a cross-workgroup hand-off access (sc1: write-through / re-fetch)
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

template <int AUX>
__device__ __forceinline__ float2 buf_ld_f2a(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, AUX));
}
template <int AUX>
__device__ __forceinline__ float buf_ld_fa(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, AUX));
}
template <int AUX>
__device__ __forceinline__ void buf_st_f2a(float2 v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    typedef int v2i __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2i, v), r, voff, soff, AUX);
}
template <int AUX>
__device__ __forceinline__ void buf_st_fa(float v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, voff, soff, AUX);
}
// a single complex element through a plain pointer: plain, or an agent-scope relaxed
// 8-byte atomic store (global_store_dwordx2 sc1)
template <int AUX>
__device__ __forceinline__ void st_c(float2* p, float2 v) {
    if constexpr (AUX == 0) *p = v;
    else __hip_atomic_store((gu64*)p, __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_u32_sc1(uint32_t* p, uint32_t v) {
    __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <int AUX>
__device__ __forceinline__ uint32_t ld_u32(const uint32_t* p) {
    if constexpr (AUX == 0) return *p;
    else return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <int AUX>
__device__ __forceinline__ float ld_f(const float* p) {
    if constexpr (AUX == 0) return *p;
    else return __builtin_bit_cast(float, __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

}  // namespace rsp
