// rsp_diag.h -- dev-only diagnostic switches of the PC / MTD kernels (rsp_kernels.hip), kept out
// of the product source.  Every switch defaults to the product build; tools/build_variant.sh
// builds a variant library with -D flags, and the A/B tools (tools/diag_pc.sh, tools/ab2.sh,
// tools/diag_stamps.py) measure it.  None of these is reachable from include/rsp.h.
//
//   -DRSP_DIAG_STAMPS          per-workgroup phase timestamps (rsp_diag_stamps export)
//   -DRSP_DIAG_PC_L2IN         PC rows read 64 L2-resident input rows (HBM reads removed)
//   -DRSP_DIAG_PC_NOSTORE      PC output stores range-checked away (HBM writes removed)
//   -DRSP_DIAG_PC_NOFFT        PC without its FFTs (load, spectrum multiply, store)
//   -DRSP_DIAG_PC_WAVES=n      minimum waves per SIMD of the PC kernel (__launch_bounds__)
//   -DRSP_DIAG_PC_LDS_EXTRA=b  extra dynamic LDS per PC workgroup (caps workgroups per CU)
//   -DRSP_MTD_NO_DMA           MTD tile loads to registers instead of LDS-DMA (the round-3 form)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rsp {

#ifdef RSP_DIAG_STAMPS
// Dev-only diagnostic build (tools/build_variant.sh, read by tools/diag_stamps.py): per-workgroup
// phase timestamps of the PC and MTD kernels.  Lane 0 of wave 0 writes the shader clock
// (s_memtime) at a phase boundary into an array no other code reads; a boundary marked `wait`
// first waits for the wave's own memory operations, so "loads arrived" / "stores done" are
// points in time.  Slots 8 and 9 hold the 100 MHz real-time clock at entry and exit; 10-12
// split the FIR (staged, computed, stored).
constexpr int kDiagSlots = 16, kDiagWG = 1 << 15;
__device__ uint64_t g_diag[2][kDiagWG * kDiagSlots];
__device__ __forceinline__ void diag_stamp(int k, int slot, bool wait, bool realtime = false) {
    if (wait) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t t = realtime ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime();
    const uint32_t wg = blockIdx.x + blockIdx.y * gridDim.x;
    if (threadIdx.x == 0 && wg < (uint32_t)kDiagWG) g_diag[k][wg * kDiagSlots + slot] = t;
}
#define RSP_STAMP(k, slot, wait) diag_stamp(k, slot, wait)
#define RSP_STAMP_RT(k, slot) diag_stamp(k, slot, false, true)
#else
#define RSP_STAMP(k, slot, wait) ((void)0)
#define RSP_STAMP_RT(k, slot) ((void)0)
#endif

#ifdef RSP_DIAG_PC_L2IN
__device__ __forceinline__ int diag_pc_src_row(int row) { return row & 63; }
#else
__device__ __forceinline__ int diag_pc_src_row(int row) { return row; }
#endif
#ifdef RSP_DIAG_PC_NOSTORE
constexpr bool kDiagPcNoStore = true;
#else
constexpr bool kDiagPcNoStore = false;
#endif
#ifdef RSP_DIAG_PC_NOFFT
constexpr bool kDiagPcNoFft = true;
#else
constexpr bool kDiagPcNoFft = false;
#endif
#ifndef RSP_DIAG_PC_WAVES
#define RSP_DIAG_PC_WAVES 2
#endif
#ifdef RSP_DIAG_PC_LDS_EXTRA
constexpr size_t kDiagPcLdsExtra = RSP_DIAG_PC_LDS_EXTRA;
#else
constexpr size_t kDiagPcLdsExtra = 0;
#endif

}  // namespace rsp
