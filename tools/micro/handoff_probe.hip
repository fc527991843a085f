// Hand-off probe for a persistent PC -> MTD dataflow on gfx950 (replaces the
// round-1 fence_cost.hip figure, which priced an agent-scope release fence -- an L2 write-back --
// per 32 KB item).  This one follows MI355X_MICROARCH.md's write-through recipe: `sc1` payload
// stores, every storing wave's asm `s_waitcnt vmcnt(0)`, a workgroup barrier, one relaxed
// agent-scope counter add per workgroup; the consumer polls the counter with an `sc1` load (one
// lane, s_sleep between polls), joins a workgroup barrier, and loads the bytes with `sc1` loads.
//
// Shape (the corner turn of one CPI, scaled): a "round" is G producer items of 32 KB (a PC row)
// followed by G consumer items that each read 32 KB / G from every producer item (an MTD tile
// reads its W columns from every row).  Each XCD has its own queue (chosen by HW_REG_XCC_ID, so
// a round's producers and consumers share one L2) and its own counters; the rounds of a queue are
// pipelined as the dataflow would be: producers of round r+1 are queued before consumers of r, and
// the payload lives in a ring of 3 slots per queue.  Per XCD the slot is 32 KB x G: G = 1 .. 128
// covers 32 KB .. 4 MB.
//
// Modes:  0 nowait   -- same items, no counters, no waits (the lower bound; data unchecked)
//         1 sc1      -- the recipe above (every word checked)
//         2 l2local  -- plain payload stores (the line stays in the XCD's L2), sc1 loads: correct
//                       only because producer and consumer are on one XCD by construction (XCC_ID)
//         3 launches -- no persistent kernel: per round one producer launch + one consumer launch
//                       over all 8 queues' items (kernel boundaries instead of counters)
// Output: us per round per queue, and the number of words a consumer saw wrong.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int kT = 256;              // threads per workgroup
constexpr int kItemF4 = 2048;        // 32 KB per item = 2048 float4
constexpr int kQ = 8;                // queues (one per XCD)
constexpr int kSlots = 3;
constexpr int kLine = 32;            // uint32 per counter line (128 B)

__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
    return v & 7u;
}

typedef int v4i __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) uint32_t gu32;
constexpr int kSc1 = 16;   // cache-policy aux bits of an sc1 (write-through / L1-bypass) access

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
template <int AUX>
__device__ __forceinline__ void st16(float4* base, int i, float4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v), rsrc(base, 0x7fffffff), (uint32_t)i * 16u, 0, AUX);
}
template <int AUX>
__device__ __forceinline__ float4 ld16(const float4* base, size_t i) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsrc(base, 0x7fffffff), (uint32_t)(i * 16u), 0, AUX));
}
__device__ __forceinline__ uint32_t ld_u32_sc1(const uint32_t* p) {
    return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct Args {
    float4* slot;        // [kQ][kSlots][G][kItemF4]
    uint32_t* ctl;       // [kQ] heads, then [kQ][kSlots][2] counters (produced, consumed), one line each
    uint32_t* bad;       // mismatching words
    uint32_t* tmo;       // a wait that timed out
    int G, rounds;
};

__device__ __forceinline__ uint32_t* head(const Args& a, int q) { return a.ctl + q * kLine; }
__device__ __forceinline__ uint32_t* ctr(const Args& a, int q, int s, int k) {
    return a.ctl + (kQ + (q * kSlots + s) * 2 + k) * kLine;
}

// thread 0: wait until *p >= target (bounded: 0.2 s, then the timeout word is set and nobody waits)
__device__ void wait_ge(const Args& a, uint32_t* p, uint32_t target) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (ld_u32_sc1(p) < target) {
        if (ld_u32_sc1(a.tmo)) return;
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {
            atomicOr(a.tmo, 1u);
            return;
        }
    }
}

__device__ __forceinline__ float4 pattern(int round, int item, int i) {
    return make_float4((float)round, (float)item, (float)i, 1.f);
}

// The item bodies carry no waits, barriers or counter adds: the loop in `flow` does those at
// fixed points with uniform control flow (a barrier under a divergent exit lets hipcc's
// structuriser sink the thread-0 counter add out of the loop body).
template <int MODE>
__device__ __forceinline__ void produce(const Args& a, int q, int r, int item) {
    float4* d = a.slot + ((size_t)(q * kSlots + r % kSlots) * a.G + item) * kItemF4;
#pragma unroll
    for (int k = 0; k < kItemF4 / kT; ++k) {
        const int i = threadIdx.x + kT * k;
        if (MODE == 1) st16<kSc1>(d, i, pattern(r, item, i));
        else st16<0>(d, i, pattern(r, item, i));
    }
}

template <int MODE>
__device__ __forceinline__ void consume(const Args& a, int q, int r, int c) {
    const float4* s = a.slot + (size_t)(q * kSlots + r % kSlots) * a.G * kItemF4;
    // consumer c reads kItemF4 / G float4 from every item: piece (item, c)
    const int per = kItemF4 / a.G;
    uint32_t badw = 0;
    float acc = 0.f;
#pragma unroll 8
    for (int k = 0; k < kItemF4 / kT; ++k) {
        const int e = threadIdx.x + kT * k;         // element of this consumer's 32 KB
        const int item = e / per, i = c * per + e % per;
        const float4 v = (MODE == 1 || MODE == 2) ? ld16<kSc1>(s, (size_t)item * kItemF4 + i) : ld16<0>(s, (size_t)item * kItemF4 + i);
        const float4 w = pattern(r, item, i);
        if (MODE != 0) badw += (v.x != w.x) + (v.y != w.y) + (v.z != w.z) + (v.w != w.w);
        acc += v.x;
    }
    if (badw) atomicAdd(a.bad, badw);
    if (acc == -1.f) a.bad[1] = 1;
}

// item k of a queue: blocks of 2G -- [G producers of round j+1][G consumers of round j] -- after
// a first block of round 0's producers
template <int MODE>
__global__ __launch_bounds__(kT) void flow(Args a) {
    __shared__ uint32_t s_item;
    const int q = (int)xcc_id();
    const uint32_t total = (uint32_t)(2 * a.rounds + 1) * a.G;   // round 0 producers + rounds blocks
    constexpr bool kSync = MODE == 1 || MODE == 2;
    for (;;) {
        // A barrier opens every iteration: without it, jump threading joins the previous item's
        // thread-0 counter add to this thread-0 claim across the back edge, the loop splits into
        // two nested loops with a divergent exit, and lanes 1-63 of wave 0 re-enter the body (and
        // its barriers) without thread 0: a hang.  A block holding a barrier (convergent) is
        // never duplicated by jump threading.
        __syncthreads();
        if (threadIdx.x == 0) s_item = __hip_atomic_fetch_add(head(a, q), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        // (wave-uniform: with the item in a VGPR the loop exit is divergent)
        const uint32_t k = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_item);
        if (k >= total) break;
        const int G = a.G;
        int kind = -1, r = 0, i = 0;   // 0 produce, 1 consume
        if (k < (uint32_t)G) {
            kind = 0, r = 0, i = (int)k;
        } else {
            const int b = (int)((k - G) / (2 * G)), o = (int)((k - G) % (2 * G));
            if (o < G) {
                if (b + 1 < a.rounds) kind = 0, r = b + 1, i = o;
            } else {
                kind = 1, r = b, i = o - G;
            }
        }
        uint32_t* wp = nullptr;
        uint32_t wt = 0;
        if (kSync && kind == 0 && r >= kSlots) wp = ctr(a, q, r % kSlots, 1), wt = (uint32_t)(r / kSlots) * G;
        if (kSync && kind == 1) wp = ctr(a, q, r % kSlots, 0), wt = (uint32_t)(r / kSlots + 1) * G;
        if (threadIdx.x == 0 && wp) wait_ge(a, wp, wt);
        __syncthreads();   // (also: every thread has read s_item)
        if (kind == 0) produce<MODE>(a, q, r, i);
        else if (kind == 1) consume<MODE>(a, q, r, i);
        if (kSync && kind >= 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (threadIdx.x == 0)
                __hip_atomic_fetch_add(ctr(a, q, r % kSlots, kind), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// which XCC each workgroup of a grid runs on (HW_REG_XCC_ID, raw bits), and whether it equals
// blockIdx.x % 8 shifted by the XCC of block 0
__global__ __launch_bounds__(kT) void xcc_census(uint32_t* hist, uint32_t* raw) {
    if (threadIdx.x == 0) {
        uint32_t v;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 16)" : "=s"(v));
        raw[blockIdx.x] = v;
        atomicAdd(hist + (v & 15u), 1u);
    }
}

__global__ __launch_bounds__(kT) void prod_launch(Args a, int r) {
    const int q = blockIdx.x / a.G, item = blockIdx.x % a.G;
    produce<3>(a, q, r, item);
}
__global__ __launch_bounds__(kT) void cons_launch(Args a, int r) {
    const int q = blockIdx.x / a.G, c = blockIdx.x % a.G;
    consume<3>(a, q, r, c);
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 64;
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int grid = cus * 4;
    const int Gs[] = {1, 8, 32, 128};
    Args a{};
    a.rounds = rounds;
    const size_t slot_bytes = (size_t)kQ * kSlots * 128 * kItemF4 * sizeof(float4);   // sized for G = 128
    hipMalloc(&a.slot, slot_bytes);
    const size_t ctl_words = (size_t)(kQ + kQ * kSlots * 2) * kLine;
    hipMalloc(&a.ctl, ctl_words * 4);
    hipMalloc(&a.bad, 8);
    hipMalloc(&a.tmo, 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    {
        uint32_t *hist, *raw;
        hipMalloc(&hist, 16 * 4);
        hipMalloc(&raw, grid * 4);
        hipMemset(hist, 0, 64);
        hipLaunchKernelGGL(xcc_census, dim3(grid), dim3(kT), 0, 0, hist, raw);
        std::vector<uint32_t> h(16), r(grid);
        hipMemcpy(h.data(), hist, 64, hipMemcpyDeviceToHost);
        hipMemcpy(r.data(), raw, grid * 4, hipMemcpyDeviceToHost);
        int match = 0;
        for (int b = 0; b < grid; ++b) match += (r[b] & 15u) == ((r[0] + b) & 7u);
        printf("XCC_ID census over %d workgroups:", grid);
        for (int i = 0; i < 16; ++i)
            if (h[i]) printf(" [%d]=%u", i, h[i]);
        printf("; raw[0..9] = %x %x %x %x %x %x %x %x %x %x; blockIdx %% 8 + XCC(0) matches %d\n", r[0], r[1], r[2], r[3],
               r[4], r[5], r[6], r[7], r[8], r[9], match);
        fflush(stdout);
    }
    printf("grid %d workgroups (%d CUs); %d rounds per queue, 8 queues; 32 KB items\n", grid, cus, rounds);
    for (int G : Gs) {
        a.G = G;
        for (int mode = 0; mode < 4; ++mode) {
            float best = 1e30f;
            uint32_t bad[2] = {0, 0}, tmo = 0;
            for (int rep = 0; rep < 3; ++rep) {
                hipMemset(a.ctl, 0, ctl_words * 4);
                hipMemset(a.bad, 0, 8);
                hipMemset(a.tmo, 0, 4);
                hipMemset(a.slot, 0xff, slot_bytes);   // stale contents: NaN words
                hipDeviceSynchronize();
                hipEventRecord(e0);
                if (mode == 0) hipLaunchKernelGGL(flow<0>, dim3(grid), dim3(kT), 0, 0, a);
                if (mode == 1) hipLaunchKernelGGL(flow<1>, dim3(grid), dim3(kT), 0, 0, a);
                if (mode == 2) hipLaunchKernelGGL(flow<2>, dim3(grid), dim3(kT), 0, 0, a);
                if (mode == 3) {
                    for (int r = 0; r < rounds; ++r) {
                        hipLaunchKernelGGL(prod_launch, dim3(kQ * G), dim3(kT), 0, 0, a, r);
                        hipLaunchKernelGGL(cons_launch, dim3(kQ * G), dim3(kT), 0, 0, a, r);
                    }
                }
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms = 0;
                hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
                uint32_t b[2], t;
                hipMemcpy(b, a.bad, 8, hipMemcpyDeviceToHost);
                hipMemcpy(&t, a.tmo, 4, hipMemcpyDeviceToHost);
                bad[0] += b[0];
                tmo |= t;
            }
            const char* names[] = {"nowait", "sc1", "l2local", "launches"};
            printf("G %3d (%5d KB per XCD slot)  %-8s  %8.2f us per round  %7.1f GB/s moved  bad words %u%s\n", G,
                   G * 32, names[mode], best * 1e3 / rounds,
                   2.0 * kQ * G * 32768.0 * rounds / (best * 1e-3) / 1e9, bad[0], tmo ? "  TIMEOUT" : "");
            fflush(stdout);
        }
    }
    return hipGetLastError() != hipSuccess;
}
