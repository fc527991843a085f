// CU-mask census and co-residency probe (VERDICT r5 item 1, step one): what a stream's CU mask
// (hipExtStreamCreateWithCUMask) bit selects on MI355X, and whether two persistent grids on two
// streams with disjoint masks are resident together (the condition a PC-only and an MTD-only
// persistent kernel need before either may spin on the other).
//
// Part 1 (census): for every mask bit b, a stream whose mask is bit b alone runs 64 one-wave
//   workgroups; each records HW_REG_XCC_ID and HW_REG_HW_ID (CU, SH, SE fields).  Printed: bit ->
//   the distinct (xcc, se, sh, cu) places its workgroups ran on; then the same for masks of 32
//   contiguous bits and of every 8th bit.
// Part 2 (co-residency): masks A = bits [0, 8 pc), B = the rest.
//   Stream A runs a grid of (CUs in A) x `per` workgroups that each spin (bounded, 1 s) until a
//   counter written by stream B's grid reaches its grid size; B's workgroups first add 1, then
//   spin until A's counter reaches A's grid.  Both complete quickly only if both grids are resident
//   at once.  Also recorded: the XCC of every workgroup of each grid (are they confined to their
//   mask's XCD slice?).
// Usage: cumask_probe [pc_per_xcd=20] [per_cu=4]
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s failed: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

typedef __attribute__((address_space(1))) uint32_t gu32;

__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
    return v;
}
__device__ __forceinline__ uint32_t hw_id() {
    uint32_t v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(v));
    return v;
}

__global__ void where_kernel(uint32_t* out) {
    if (threadIdx.x == 0) {
        out[blockIdx.x * 2 + 0] = xcc_id();
        out[blockIdx.x * 2 + 1] = hw_id();
    }
}

__device__ __forceinline__ uint32_t ld_sc1(const uint32_t* p) {
    return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// every workgroup: add 1 to mine, wait until other >= target (bounded 1 s), record where it ran
__global__ void meet_kernel(uint32_t* mine, const uint32_t* other, uint32_t target, uint32_t* tmo, uint32_t* place,
                            unsigned long long* t_done) {
    if (threadIdx.x == 0) {
        place[blockIdx.x] = xcc_id() | (hw_id() << 8) ;
        __hip_atomic_fetch_add((gu32*)mine, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (ld_sc1(other) < target) {
            __builtin_amdgcn_s_sleep(4);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {   // 1 s of the 100 MHz clock
                __hip_atomic_fetch_or((gu32*)tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        t_done[blockIdx.x] = __builtin_amdgcn_s_memrealtime() - t0;
    }
    __syncthreads();
}

int main(int argc, char** argv) {
    const int pc = argc > 1 ? atoi(argv[1]) : 20;
    const int per = argc > 2 ? atoi(argv[2]) : 4;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int ncu = prop.multiProcessorCount;
    const int words = (ncu + 31) / 32;
    printf("device %s, %d CUs, mask words %d\n", prop.gcnArchName, ncu, words);
    uint32_t* d_out;
    constexpr int kWG = 64;   // workgroups per census launch (dealt over the XCDs)
    CK(hipMalloc(&d_out, kWG * 2 * 4));
    std::vector<int> bit_xcc(ncu, -1), bit_cu(ncu, -1), bit_se(ncu, -1), bit_sh(ncu, -1);
    // census of a mask: the distinct (xcc, se, sh, cu) places of kWG workgroups
    auto census = [&](const std::vector<uint32_t>& mask, std::vector<uint32_t>& places) {
        hipStream_t s;
        CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask.data()));
        CK(hipMemsetAsync(d_out, 0xff, kWG * 2 * 4, s));
        hipLaunchKernelGGL(where_kernel, dim3(kWG), dim3(64), 0, s, d_out);
        CK(hipGetLastError());
        uint32_t h[kWG * 2];
        CK(hipMemcpyAsync(h, d_out, sizeof(h), hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        CK(hipStreamDestroy(s));
        places.clear();
        for (int i = 0; i < kWG; ++i) {
            // HW_ID (gfx9 layout): wave 3:0, simd 5:4, pipe 7:6, cu 11:8, sh 12, se 15:13
            const uint32_t x = h[2 * i] & 0xf, hid = h[2 * i + 1];
            const uint32_t key = (x << 12) | (((hid >> 13) & 7) << 8) | (((hid >> 12) & 1) << 4) | ((hid >> 8) & 0xf);
            bool seen = false;
            for (uint32_t p : places) seen |= p == key;
            if (!seen) places.push_back(key);
        }
    };
    int disagree = 0;
    printf("census: per single-bit mask, the distinct places (xcc:se.sh.cu) of %d workgroups\n", kWG);
    std::vector<uint32_t> pl;
    for (int b = 0; b < ncu; ++b) {
        std::vector<uint32_t> mask(words, 0u);
        mask[b / 32] = 1u << (b % 32);
        census(mask, pl);
        if (pl.size() != 1) ++disagree;
        const uint32_t k = pl[0];
        bit_xcc[b] = (int)(k >> 12);
        bit_se[b] = (int)((k >> 8) & 7);
        bit_sh[b] = (int)((k >> 4) & 1);
        bit_cu[b] = (int)(k & 0xf);
        printf("%3d:", b);
        for (size_t i = 0; i < pl.size() && i < 8; ++i)
            printf(" %u:%u.%u.%u", pl[i] >> 12, (pl[i] >> 8) & 7, (pl[i] >> 4) & 1, pl[i] & 0xf);
        printf("%s\n", pl.size() > 8 ? " ..." : "");
    }
    printf("single-bit masks whose workgroups used more than one place: %d of %d\n", disagree, ncu);
    for (int g = 0; g < ncu / 32; ++g) {
        std::vector<uint32_t> mask(words, 0u);
        mask[g] = 0xffffffffu;
        census(mask, pl);
        int per[8] = {};
        for (uint32_t p : pl) ++per[(p >> 12) & 7];
        printf("mask bits [%d, %d): %zu places; per xcc:", 32 * g, 32 * g + 32, pl.size());
        for (int x = 0; x < 8; ++x) printf(" %d", per[x]);
        printf("\n");
    }
    {   // bits b with b % 8 == r
        for (int r = 0; r < 8; r += 7) {
            std::vector<uint32_t> mask(words, 0u);
            for (int b = r; b < ncu; b += 8) mask[b / 32] |= 1u << (b % 32);
            census(mask, pl);
            int per[8] = {};
            for (uint32_t p : pl) ++per[(p >> 12) & 7];
            printf("mask bits = %d mod 8: %zu places; per xcc:", r, pl.size());
            for (int x = 0; x < 8; ++x) printf(" %d", per[x]);
            printf("\n");
        }
    }

    // Part 2: co-residency of two spinning grids with disjoint masks, `pc` CUs per XCD in A
    std::vector<uint32_t> mA(words, 0u), mB(words, 0u);
    int nA = 0, nB = 0;
    for (int b = 0; b < ncu; ++b) {   // A = bits [0, 8 * pc), B = the rest
        if (b < 8 * pc) {
            mA[b / 32] |= 1u << (b % 32);
            ++nA;
        } else {
            mB[b / 32] |= 1u << (b % 32);
            ++nB;
        }
    }
    hipStream_t sA, sB;
    CK(hipExtStreamCreateWithCUMask(&sA, (uint32_t)words, mA.data()));
    CK(hipExtStreamCreateWithCUMask(&sB, (uint32_t)words, mB.data()));
    uint32_t* d_ctl;
    CK(hipMalloc(&d_ctl, 3 * 128));
    const int gA = nA * per, gB = nB * per;
    uint32_t *d_pA, *d_pB;
    unsigned long long *d_tA, *d_tB;
    CK(hipMalloc(&d_pA, gA * 4));
    CK(hipMalloc(&d_pB, gB * 4));
    CK(hipMalloc(&d_tA, gA * 8));
    CK(hipMalloc(&d_tB, gB * 8));
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipMemset(d_ctl, 0, 3 * 128));
        CK(hipDeviceSynchronize());
        uint32_t* cA = d_ctl;
        uint32_t* cB = d_ctl + 32;
        uint32_t* tmo = d_ctl + 64;
        hipLaunchKernelGGL(meet_kernel, dim3(gA), dim3(256), 0, sA, cA, cB, (uint32_t)gB, tmo, d_pA, d_tA);
        hipLaunchKernelGGL(meet_kernel, dim3(gB), dim3(256), 0, sB, cB, cA, (uint32_t)gA, tmo, d_pB, d_tB);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        uint32_t h[3 * 32];
        CK(hipMemcpy(h, d_ctl, sizeof(h), hipMemcpyDeviceToHost));
        std::vector<uint32_t> pA(gA), pB(gB);
        std::vector<unsigned long long> tA(gA), tB(gB);
        CK(hipMemcpy(pA.data(), d_pA, gA * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(pB.data(), d_pB, gB * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(tA.data(), d_tA, gA * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(tB.data(), d_tB, gB * 8, hipMemcpyDeviceToHost));
        std::vector<int> xa(8, 0), xb(8, 0);
        int strayA = 0, strayB = 0;
        for (int i = 0; i < gA; ++i) {
            ++xa[pA[i] & 7];
            // the workgroup's (xcc, se, sh, cu) must be one of mask A's
            const uint32_t hid = pA[i] >> 8;
            bool ok = false;
            for (int b = 0; b < ncu && !ok; ++b)
                ok = (mA[b / 32] >> (b % 32) & 1u) && bit_xcc[b] == (int)(pA[i] & 0xf) && bit_cu[b] == (int)((hid >> 8) & 0xf) &&
                     bit_sh[b] == (int)((hid >> 12) & 1) && bit_se[b] == (int)((hid >> 13) & 7);
            strayA += !ok;
        }
        for (int i = 0; i < gB; ++i) {
            ++xb[pB[i] & 7];
            const uint32_t hid = pB[i] >> 8;
            bool ok = false;
            for (int b = 0; b < ncu && !ok; ++b)
                ok = (mB[b / 32] >> (b % 32) & 1u) && bit_xcc[b] == (int)(pB[i] & 0xf) && bit_cu[b] == (int)((hid >> 8) & 0xf) &&
                     bit_sh[b] == (int)((hid >> 12) & 1) && bit_se[b] == (int)((hid >> 13) & 7);
            strayB += !ok;
        }
        unsigned long long mxA = 0, mxB = 0;
        for (auto t : tA) mxA = t > mxA ? t : mxA;
        for (auto t : tB) mxB = t > mxB ? t : mxB;
        printf("co-residency rep %d: A %d CUs x %d = %d WGs, B %d CUs x %d = %d WGs; counters %u / %u; timeout %u; "
               "max wait A %.1f us, B %.1f us; stray A %d, B %d\n",
               rep, nA, per, gA, nB, per, gB, h[0], h[32], h[64], mxA / 100.0, mxB / 100.0, strayA, strayB);
        printf("  A per xcc:");
        for (int x = 0; x < 8; ++x) printf(" %d", xa[x]);
        printf("   B per xcc:");
        for (int x = 0; x < 8; ++x) printf(" %d", xb[x]);
        printf("\n");
    }
    CK(hipStreamDestroy(sA));
    CK(hipStreamDestroy(sB));
    return 0;
}
