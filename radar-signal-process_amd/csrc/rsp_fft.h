// rsp_fft.h -- in-LDS mixed-radix Stockham FFT building blocks for gfx950.
//
// A length-N complex fp32 FFT lives in one LDS array (float2, one pad slot per 16
// elements so the stride-R scatter of a radix-R pass is bank-conflict free).  Each pass
// is the autosorting Stockham DIT step (Govindaraju et al., SC'08):
//     for butterfly j < N/R:  v[r] = buf[j + r*N/R] * W_{Ns*R}^{r*(j%Ns)};  v = DFT_R(v);
//                             buf[(j/Ns)*Ns*R + j%Ns + r*Ns] = v[r]
// done in place: every thread reads its R inputs to registers, a barrier, then writes.
// The radix plan is chosen at compile time (largest of 16/8/4/2 with N/R >= the threads
// working on one transform, radix 3 for the 3*2^k sizes), so every index division is by
// a compile-time constant.  Twiddles come from a per-N fp32 table W_N^e built in fp64 on
// the host (accurate to 0.5 ulp), read through the vector L1/L2.
#pragma once
#include <hip/hip_runtime.h>

namespace rsp {

__device__ __forceinline__ float2 cconj(float2 a) { return make_float2(a.x, -a.y); }
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }

// Packed-FP32 complex primitives.  gfx950's VOP3P v_pk_* instructions take per-half
// operand selects (op_sel / op_sel_hi) and negations (neg_lo / neg_hi), so a (+-j) rotation
// folded into an add, or a complex product, needs no register shuffles.  hipcc does not
// emit the negation modifiers on its own (it spends v_xor + v_mov per rotation), hence the
// inline asm; -DRSP_NO_ASM selects the portable forms.
#ifndef RSP_NO_ASM
// Plain add/sub as 2-wide vector arithmetic: one v_pk_add_f32 each (the subtraction's
// negation folds into neg_lo/neg_hi).  Written on scalar halves, the SLP vectorizer pairs
// lanes of *different* complex values and shuffles them back with v_mov; written as asm,
// every dependent pair of statements costs an s_nop (see cmul).
typedef float v2f __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float2 cadd(float2 a, float2 b) {
    return __builtin_bit_cast(float2, __builtin_bit_cast(v2f, a) + __builtin_bit_cast(v2f, b));
}
__device__ __forceinline__ float2 csub(float2 a, float2 b) {
    return __builtin_bit_cast(float2, __builtin_bit_cast(v2f, a) - __builtin_bit_cast(v2f, b));
}
// a + (-j) b = (a.x + b.y, a.y - b.x): one v_pk_fma_f32 of the swapped b times (1, -1) --
// the products by +-1 are exact, so the fma rounds exactly as the add (the constant pair
// lives in SGPRs; hipcc does not fold a per-half negation into neg_lo/neg_hi itself).
__device__ __forceinline__ float2 add_mj(float2 a, float2 b) {
    const v2f bs = __builtin_shufflevector(__builtin_bit_cast(v2f, b), __builtin_bit_cast(v2f, b), 1, 0);
    return __builtin_bit_cast(float2, __builtin_elementwise_fma(bs, (v2f){1.f, -1.f}, __builtin_bit_cast(v2f, a)));
}
// a + j b = (a.x - b.y, a.y + b.x)
__device__ __forceinline__ float2 add_pj(float2 a, float2 b) {
    const v2f bs = __builtin_shufflevector(__builtin_bit_cast(v2f, b), __builtin_bit_cast(v2f, b), 1, 0);
    return __builtin_bit_cast(float2, __builtin_elementwise_fma(bs, (v2f){-1.f, 1.f}, __builtin_bit_cast(v2f, a)));
}
// a * b in two instructions: m = (-a.y b.y, a.y b.x); d = (a.x b.x, a.x b.y) + m
// (hipcc builds m from a negated copy and a v_mov shuffle: four instructions)
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    float2 m, d;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0] neg_lo:[1,0]" : "=v"(m) : "v"(a), "v"(b));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(d) : "v"(a), "v"(b), "v"(m));
    return d;
}
// conj(a * b) in two instructions (negated high half of the fma)
__device__ __forceinline__ float2 cmul_conj(float2 a, float2 b) {
    float2 m, d;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0] neg_lo:[1,0]" : "=v"(m) : "v"(a), "v"(b));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] neg_hi:[1,0,1]" : "=v"(d) : "v"(a), "v"(b), "v"(m));
    return d;
}
// Two independent complex products in one asm statement, interleaved (mul0 mul1 fma0 fma1):
// gfx950 needs one wait state between a packed-FP32 result and a VALU that reads it, which
// hipcc pays as an s_nop after every asm statement whose result the next one reads -- 245 of
// the PC kernel's 418 nops sat inside cmul.  Interleaved, each fma is one instruction behind
// its mul.  m0, m1, d0 are early-clobber (written before the inputs' last reads).
__device__ __forceinline__ void cmul2(float2& d0, float2 a0, float2 b0, float2& d1, float2 a1, float2 b1) {
    float2 m0, m1, e0, e1;
    asm("v_pk_mul_f32 %2, %4, %5 op_sel:[1,1] op_sel_hi:[1,0] neg_lo:[1,0]\n\t"
        "v_pk_mul_f32 %3, %6, %7 op_sel:[1,1] op_sel_hi:[1,0] neg_lo:[1,0]\n\t"
        "v_pk_fma_f32 %0, %4, %5, %2 op_sel_hi:[0,1,1]\n\t"
        "v_pk_fma_f32 %1, %6, %7, %3 op_sel_hi:[0,1,1]"
        : "=&v"(e0), "=v"(e1), "=&v"(m0), "=&v"(m1)
        : "v"(a0), "v"(b0), "v"(a1), "v"(b1));
    d0 = e0;
    d1 = e1;
}
// conj(a0 * b0), conj(a1 * b1), as cmul2
__device__ __forceinline__ void cmul2_conj(float2& d0, float2 a0, float2 b0, float2& d1, float2 a1, float2 b1) {
    float2 m0, m1, e0, e1;
    asm("v_pk_mul_f32 %2, %4, %5 op_sel:[1,1] op_sel_hi:[1,0] neg_lo:[1,0]\n\t"
        "v_pk_mul_f32 %3, %6, %7 op_sel:[1,1] op_sel_hi:[1,0] neg_lo:[1,0]\n\t"
        "v_pk_fma_f32 %0, %4, %5, %2 op_sel_hi:[0,1,1] neg_hi:[1,0,1]\n\t"
        "v_pk_fma_f32 %1, %6, %7, %3 op_sel_hi:[0,1,1] neg_hi:[1,0,1]"
        : "=&v"(e0), "=v"(e1), "=&v"(m0), "=&v"(m1)
        : "v"(a0), "v"(b0), "v"(a1), "v"(b1));
    d0 = e0;
    d1 = e1;
}
#else
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 add_mj(float2 a, float2 b) { return make_float2(a.x + b.y, a.y - b.x); }
__device__ __forceinline__ float2 add_pj(float2 a, float2 b) { return make_float2(a.x - b.y, a.y + b.x); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(fmaf(a.x, b.x, -a.y * b.y), fmaf(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ float2 cmul_conj(float2 a, float2 b) { return cconj(cmul(a, b)); }
__device__ __forceinline__ void cmul2(float2& d0, float2 a0, float2 b0, float2& d1, float2 a1, float2 b1) {
    d0 = cmul(a0, b0);
    d1 = cmul(a1, b1);
}
__device__ __forceinline__ void cmul2_conj(float2& d0, float2 a0, float2 b0, float2& d1, float2 a1, float2 b1) {
    d0 = cmul_conj(a0, b0);
    d1 = cmul_conj(a1, b1);
}
#endif
// a * (-j)
__device__ __forceinline__ float2 cmul_mj(float2 a) { return make_float2(a.y, -a.x); }

// LDS index with one pad slot per 16 elements.
__host__ __device__ constexpr int pidx(int i) { return i + (i >> 4); }
__host__ __device__ constexpr int padded_len(int n) { return n + (n >> 4) + 1; }

// ---------------------------------------------------------------- register DFTs (forward)
__device__ __forceinline__ void dft2(float2& a, float2& b) {
    float2 t = a;
    a = cadd(t, b);
    b = csub(t, b);
}

__device__ __forceinline__ void dft4(float2& a0, float2& a1, float2& a2, float2& a3) {
    const float2 t0 = cadd(a0, a2), t1 = csub(a0, a2);
    const float2 t2 = cadd(a1, a3), d = csub(a1, a3);
    a0 = cadd(t0, t2);
    a2 = csub(t0, t2);
    a1 = add_mj(t1, d);   // t1 + (-j) d
    a3 = add_pj(t1, d);   // t1 - (-j) d
}

// DFT4 of (a0, a1, -j*a2, a3): the W16^4 = -j twiddle folded into the first butterfly
__device__ __forceinline__ void dft4_a2mj(float2& a0, float2& a1, float2& a2, float2& a3) {
    const float2 t0 = add_mj(a0, a2), t1 = add_pj(a0, a2);
    const float2 t2 = cadd(a1, a3), d = csub(a1, a3);
    a0 = cadd(t0, t2);
    a2 = csub(t0, t2);
    a1 = add_mj(t1, d);
    a3 = add_pj(t1, d);
}

__device__ __forceinline__ void dft3(float2& a0, float2& a1, float2& a2) {
    const float s = 0.86602540378443864676f;  // sqrt(3)/2
    float2 t = cadd(a1, a2);
    float2 d = csub(a1, a2);
    float2 m = make_float2(a0.x - 0.5f * t.x, a0.y - 0.5f * t.y);
    a0 = cadd(a0, t);
    // X1 = m - j*s*d ; X2 = m + j*s*d
    float2 jd = make_float2(-s * d.y, s * d.x);  // j*s*d
    a1 = csub(m, jd);
    a2 = cadd(m, jd);
}

__device__ __forceinline__ void dft8(float2* v) {
    const float h = 0.70710678118654752440f;
    float2 e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6];
    float2 o0 = v[1], o1 = v[3], o2 = v[5], o3 = v[7];
    dft4(e0, e1, e2, e3);
    dft4(o0, o1, o2, o3);
    // o_k *= W8^k (W8^2 = -j folded into the adds)
    cmul2(o1, o1, make_float2(h, -h), o3, o3, make_float2(-h, -h));
    v[0] = cadd(e0, o0); v[4] = csub(e0, o0);
    v[1] = cadd(e1, o1); v[5] = csub(e1, o1);
    v[2] = add_mj(e2, o2); v[6] = add_pj(e2, o2);
    v[3] = cadd(e3, o3); v[7] = csub(e3, o3);
}

__device__ __forceinline__ void dft16(float2* v) {
    // n = 4*n1 + n2, k = k1 + 4*k2
    const float c1 = 0.92387953251128675613f, s1 = 0.38268343236508977173f;
    const float h = 0.70710678118654752440f;
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) dft4(v[n2], v[4 + n2], v[8 + n2], v[12 + n2]);
    // v[4*k1 + n2] now holds b[n2][k1]; multiply by W16^(n2*k1)
    // n2=1: k1=1..3 -> W^1, W^2, W^3 ; n2=2: W^2, W^4, W^6 ; n2=3: W^3, W^6, W^9
    cmul2(v[5], v[5], make_float2(c1, -s1), v[9], v[9], make_float2(h, -h));
    cmul2(v[13], v[13], make_float2(s1, -c1), v[6], v[6], make_float2(h, -h));
    // v[10] *= W16^4 = -j: folded into dft4_a2mj below
    cmul2(v[14], v[14], make_float2(-h, -h), v[7], v[7], make_float2(s1, -c1));
    cmul2(v[11], v[11], make_float2(-h, -h), v[15], v[15], make_float2(-c1, s1));
    // second stage: for each k1, DFT4 over n2 of v[4*k1 + n2] -> X[k1 + 4*k2]
    float2 x[16];
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) {
        float2 a0 = v[4 * k1 + 0], a1 = v[4 * k1 + 1], a2 = v[4 * k1 + 2], a3 = v[4 * k1 + 3];
        if (k1 == 2) dft4_a2mj(a0, a1, a2, a3);
        else dft4(a0, a1, a2, a3);
        x[k1] = a0; x[k1 + 4] = a1; x[k1 + 8] = a2; x[k1 + 12] = a3;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = x[i];
}

template <int R>
__device__ __forceinline__ void dft(float2* v) {
    if constexpr (R == 2) {
        dft2(v[0], v[1]);
    } else if constexpr (R == 3) {
        dft3(v[0], v[1], v[2]);
    } else if constexpr (R == 4) {
        dft4(v[0], v[1], v[2], v[3]);
    } else if constexpr (R == 8) {
        dft8(v);
    } else if constexpr (R == 16) {
        dft16(v);
    } else {
        static_assert(R == 2, "unsupported radix");
    }
}

// ---------------------------------------------------------------- plan + passes
__host__ __device__ constexpr int pick_radix(int rem, int n, int g) {
    // prefer the largest power-of-two radix that keeps every working thread busy
    if (rem % 16 == 0 && n / 16 >= g) return 16;
    if (rem % 8 == 0 && n / 8 >= g) return 8;
    if (rem % 4 == 0 && n / 4 >= g) return 4;
    if (rem % 16 == 0) return 16;
    if (rem % 8 == 0) return 8;
    if (rem % 4 == 0) return 4;
    if (rem % 2 == 0) return 2;
    if (rem % 3 == 0) return 3;
    return rem;
}

__host__ __device__ constexpr bool fft_size_ok(int n) {
    if (n < 2) return false;
    while (n % 2 == 0) n /= 2;
    return n == 1 || n == 3;
}

// One Stockham pass.  G threads (t = 0..G-1) work on this transform; other threads of the
// block must call with t >= G so the barriers stay uniform.
template <int N, int R, int G, int Ns>
__device__ __forceinline__ void fft_pass(float2* buf, int t, const float2* __restrict__ tw) {
    constexpr int NB = N / R;
    constexpr int PER = (NB + G - 1) / G;
    float2 v[PER][R];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int j = t + i * G;
        if (t < G && j < NB) {
#pragma unroll
            for (int r = 0; r < R; ++r) v[i][r] = buf[pidx(j + r * NB)];
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int j = t + i * G;
        if (t < G && j < NB) {
            const int k = j % Ns;
            if constexpr (Ns > 1) {
                constexpr int STRIDE = N / (Ns * R);
                const int e = k * STRIDE;
#pragma unroll
                for (int r = 1; r < R; ++r) v[i][r] = cmul(v[i][r], tw[r * e]);
            }
            dft<R>(v[i]);
            const int idxD = (j / Ns) * Ns * R + k;
#pragma unroll
            for (int r = 0; r < R; ++r) buf[pidx(idxD + r * Ns)] = v[i][r];
        }
    }
    __syncthreads();
}

template <int N, int G, int Ns>
__device__ __forceinline__ void fft_rec(float2* buf, int t, const float2* __restrict__ tw) {
    if constexpr (Ns < N) {
        constexpr int R = pick_radix(N / Ns, N, G);
        static_assert(R == 2 || R == 3 || R == 4 || R == 8 || R == 16, "FFT size must be 2^k or 3*2^k");
        fft_pass<N, R, G, Ns>(buf, t, tw);
        fft_rec<N, G, Ns * R>(buf, t, tw);
    }
}

// Forward FFT (e^{-i}) of buf[pidx(0..N-1)], natural order in and out, in place.
// Every thread of the block must call it (it contains barriers).
template <int N, int G>
__device__ __forceinline__ void fft_lds(float2* buf, int t, const float2* __restrict__ tw) {
    fft_rec<N, G, 1>(buf, t, tw);
}

// ---------------------------------------------------------------- register-resident FFT
// G threads share one length-N transform; thread t holds E = N/G elements in the
// "strided" pattern u[m] = x[t + G*m].  Every Stockham pass with radix R | E gives each
// thread PER = E/R butterflies j = t + i*G whose inputs are x[j + r*N/R] = u[i + r*PER],
// so the first pass reads straight from registers (no LDS) and the last pass leaves
// X[t + G*m] in u[m] -- natural order, coalesced for global stores, and exactly the input
// pattern of the next transform (forward FFT -> spectrum multiply -> inverse FFT never
// touches LDS in between).  Intermediate passes exchange through `buf` (N padded slots).
__host__ __device__ constexpr int pick_radix_e(int rem, int e) {
    if (rem % 16 == 0 && e % 16 == 0) return 16;
    if (rem % 8 == 0 && e % 8 == 0) return 8;
    if (rem % 4 == 0 && e % 4 == 0) return 4;
    if (rem % 2 == 0 && e % 2 == 0) return 2;
    if (rem % 3 == 0 && e % 3 == 0) return 3;
    return 0;
}

// LDS slot of element (base + r*S) for r < R: affine in r whenever the padding allows it
// (S a multiple of 16, or S == 1 with R | 16 and R | base), so the compiler emits one
// address register and immediate offsets instead of R live addresses.
template <int S, int R>
__device__ __forceinline__ int slot(int base, int r) {
    if constexpr (S % 16 == 0) return pidx(base) + r * (S + S / 16);
    else if constexpr (S == 1 && 16 % R == 0) return pidx(base) + r;   // base is a multiple of R
    else return pidx(base + r * S);
}

// v[r] *= W^(r*e) for r = 1..R-1, W = e^{-2 pi i/N}, from the fp32 table tw[0..N).
// Radix 16 reads 6 table entries (W^e, W^2e, W^3e, W^4e, W^8e, W^12e) and forms the rest
// with one complex product each (~1.5 ulp), instead of 15 gathers.
template <int R, int N>
__device__ __forceinline__ void twiddle(float2* v, int e, const float2* __restrict__ tw) {
    if constexpr (R == 16) {
        const float2 w1 = tw[e], w2 = tw[2 * e], w3 = tw[3 * e];
        const float2 w4 = tw[4 * e], w8 = tw[8 * e], w12 = tw[12 * e];
        v[1] = cmul(v[1], w1);
        v[2] = cmul(v[2], w2);
        v[3] = cmul(v[3], w3);
        v[4] = cmul(v[4], w4);
        v[5] = cmul(v[5], cmul(w4, w1));
        v[6] = cmul(v[6], cmul(w4, w2));
        v[7] = cmul(v[7], cmul(w4, w3));
        v[8] = cmul(v[8], w8);
        v[9] = cmul(v[9], cmul(w8, w1));
        v[10] = cmul(v[10], cmul(w8, w2));
        v[11] = cmul(v[11], cmul(w8, w3));
        v[12] = cmul(v[12], w12);
        v[13] = cmul(v[13], cmul(w12, w1));
        v[14] = cmul(v[14], cmul(w12, w2));
        v[15] = cmul(v[15], cmul(w12, w3));
    } else if constexpr (R == 8) {
        const float2 w1 = tw[e], w2 = tw[2 * e], w3 = tw[3 * e], w4 = tw[4 * e];
        v[1] = cmul(v[1], w1);
        v[2] = cmul(v[2], w2);
        v[3] = cmul(v[3], w3);
        v[4] = cmul(v[4], w4);
        v[5] = cmul(v[5], cmul(w4, w1));
        v[6] = cmul(v[6], cmul(w4, w2));
        v[7] = cmul(v[7], cmul(w4, w3));
    } else {
#pragma unroll
        for (int r = 1; r < R; ++r) v[r] = cmul(v[r], tw[r * e]);
    }
}

template <int N, int G, int Ns, int E>
__device__ __forceinline__ void fft_reg(float2 (&u)[E], float2* buf, int t, const float2* __restrict__ tw) {
    if constexpr (Ns < N) {
        constexpr int R = pick_radix_e(N / Ns, E);
        static_assert(R != 0, "no radix divides both the remaining length and E");
        constexpr int NB = N / R;
        constexpr int PER = E / R;
        static_assert(NB == PER * G, "thread count and radix plan disagree");
        if constexpr (Ns > 1) {
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int b = t + i * G;
#pragma unroll
                for (int r = 0; r < R; ++r) u[i + r * PER] = buf[slot<NB, R>(b, r)];
            }
        }
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            float2 v[R];
#pragma unroll
            for (int r = 0; r < R; ++r) v[r] = u[i + r * PER];
            if constexpr (Ns > 1) {
                const int k = (t + i * G) % Ns;
                twiddle<R, N>(v, k * (N / (Ns * R)), tw);
            }
            dft<R>(v);
#pragma unroll
            for (int r = 0; r < R; ++r) u[i + r * PER] = v[r];
        }
        if constexpr (Ns * R < N) {
            __syncthreads();  // WAR: earlier readers of buf are done
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int j = t + i * G;
                const int base = (j / Ns) * Ns * R + (j % Ns);
#pragma unroll
                for (int r = 0; r < R; ++r) buf[slot<Ns, R>(base, r)] = u[i + r * PER];
            }
            __syncthreads();  // RAW
        }
        fft_reg<N, G, Ns * R, E>(u, buf, t, tw);
    }
}


// ---------------------------------------------------------------- preloaded twiddles
// The inverse transform is conj(FFT(conj(.))), so forward and inverse passes use the
// same twiddle entries: a thread loads its per-pass twiddles once (tw_preload, issued
// together with the row's input loads so their latency overlaps) and every pass reads
// them from registers instead of waiting on table loads after each LDS exchange.
//
// Lean twiddles: a thread keeps only the base twiddles W^e (and W^4e for radix 8/16) of each
// butterfly and forms the other powers with complex products when it applies them (radix 16:
// W^2e = (W^e)^2, W^3e, W^8e = (W^4e)^2, W^12e; ~2-4 ulp) -- 8 VGPRs instead of 24 for a
// 4096-point row of E = 16, so more rows stay resident per SIMD.
__host__ __device__ constexpr int tw_loads(int R) { return R >= 8 ? 2 : 1; }

template <int N, int E>
__host__ __device__ constexpr int tw_regs(int Ns = 1) {
    int total = 0;
    while (Ns < N) {
        const int R = pick_radix_e(N / Ns, E);
        if (Ns > 1) total += (E / R) * tw_loads(R);
        Ns *= R;
    }
    return total;
}

template <int R>
__device__ __forceinline__ void tw_fetch(float2* w, int e, const float2* __restrict__ tw) {
    w[0] = tw[e];
    if constexpr (R >= 8) w[1] = tw[4 * e];
}

// v[r] *= W^(r*e) from the tw_fetch<R> entries (same products as twiddle<R, N>)
template <int R>
__device__ __forceinline__ void tw_apply(float2* v, const float2* w) {
    if constexpr (R == 16) {
        // opaque copies: the derived powers are formed at every use instead of being hoisted
        // out of a row loop into registers (which would undo the saving)
        float2 w1 = w[0], w4 = w[1];
        asm volatile("" : "+v"(w1), "+v"(w4));
        // the same products as before, paired so each pair's inputs were formed >= 1 pair earlier
        float2 w2, w3, w8, w12, p5, p6, p7, p9, p10, p11, p13, p14, p15;
        cmul2(w2, w1, w1, w8, w4, w4);
        cmul2(w3, w2, w1, w12, w8, w4);
        cmul2(v[1], v[1], w1, v[2], v[2], w2);
        cmul2(v[3], v[3], w3, p5, w4, w1);
        cmul2(v[4], v[4], w4, p6, w4, w2);
        cmul2(v[5], v[5], p5, p7, w4, w3);
        cmul2(v[6], v[6], p6, p9, w8, w1);
        cmul2(v[7], v[7], p7, p10, w8, w2);
        cmul2(v[8], v[8], w8, p11, w8, w3);
        cmul2(v[9], v[9], p9, p13, w12, w1);
        cmul2(v[10], v[10], p10, p14, w12, w2);
        cmul2(v[11], v[11], p11, p15, w12, w3);
        cmul2(v[12], v[12], w12, v[13], v[13], p13);
        cmul2(v[14], v[14], p14, v[15], v[15], p15);
    } else if constexpr (R == 8) {
        float2 w1 = w[0], w4 = w[1];
        asm volatile("" : "+v"(w1), "+v"(w4));
        float2 w2, w3, p5, p6, p7;
        cmul2(w2, w1, w1, p5, w4, w1);
        cmul2(w3, w2, w1, v[1], v[1], w1);
        cmul2(v[2], v[2], w2, p6, w4, w2);
        cmul2(v[3], v[3], w3, p7, w4, w3);
        cmul2(v[4], v[4], w4, v[5], v[5], p5);
        cmul2(v[6], v[6], p6, v[7], v[7], p7);
    } else {
        float2 w0 = w[0];
        asm volatile("" : "+v"(w0));
        float2 wr = w0;
#pragma unroll
        for (int r = 1; r < R; ++r) {
            v[r] = cmul(v[r], wr);
            if (r + 1 < R) wr = cmul(wr, w0);
        }
    }
}

template <int N, int G, int Ns, int E, int WO, int NW>
__device__ __forceinline__ void tw_preload(float2 (&w)[NW], int t, const float2* __restrict__ tw) {
    if constexpr (Ns < N) {
        constexpr int R = pick_radix_e(N / Ns, E);
        constexpr int PER = E / R;
        constexpr int L = tw_loads(R);
        if constexpr (Ns > 1) {
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int k = (t + i * G) % Ns;
                tw_fetch<R>(w + WO + i * L, k * (N / (Ns * R)), tw);
            }
        }
        tw_preload<N, G, Ns * R, E, WO + (Ns > 1 ? PER * L : 0), NW>(w, t, tw);
    }
}

// fft_reg with the twiddles of every pass already in registers (w from tw_preload)
// Exchange synchronisation: the workgroup barrier, or (WS: the transform belongs to one wave)
// a wave-scope fence -- a wave's LDS operations are performed in issue order.
// Workgroup barrier for an LDS hand-off: this wave's LDS operations complete, then s_barrier.
// __syncthreads() is a workgroup-scope release/acquire fence around the barrier, and once a
// kernel has issued an LDS-DMA load (the MTD tile) hipcc makes every such fence wait vmcnt(0) --
// for every global load and store the wave has in flight, e.g. the range job's gathers or the
// RDM stores -- although only LDS changes hands here.  (The "memory" clobber keeps hipcc from
// moving memory accesses across it.)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <bool WS>
__device__ __forceinline__ void xsync() {
    if constexpr (WS) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
        lds_barrier();
    }
}

template <int N, int G, int Ns, int E, int WO, int NW, bool WS = false>
__device__ __forceinline__ void fft_reg_w(float2 (&u)[E], float2* buf, int t, const float2 (&w)[NW]) {
    if constexpr (Ns < N) {
        constexpr int R = pick_radix_e(N / Ns, E);
        static_assert(R != 0, "no radix divides both the remaining length and E");
        constexpr int NB = N / R;
        constexpr int PER = E / R;
        constexpr int L = tw_loads(R);
        static_assert(NB == PER * G, "thread count and radix plan disagree");
        if constexpr (Ns > 1) {
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int b = t + i * G;
#pragma unroll
                for (int r = 0; r < R; ++r) u[i + r * PER] = buf[slot<NB, R>(b, r)];
            }
        }
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            float2 v[R];
#pragma unroll
            for (int r = 0; r < R; ++r) v[r] = u[i + r * PER];
            if constexpr (Ns > 1) tw_apply<R>(v, w + WO + i * L);
            dft<R>(v);
#pragma unroll
            for (int r = 0; r < R; ++r) u[i + r * PER] = v[r];
        }
        if constexpr (Ns * R < N) {
            xsync<WS>();  // WAR: earlier readers of buf are done
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int j = t + i * G;
                const int base = (j / Ns) * Ns * R + (j % Ns);
#pragma unroll
                for (int r = 0; r < R; ++r) buf[slot<Ns, R>(base, r)] = u[i + r * PER];
            }
            xsync<WS>();  // RAW
        }
        fft_reg_w<N, G, Ns * R, E, WO + (Ns > 1 ? PER * L : 0), NW, WS>(u, buf, t, w);
    }
}

// ---------------------------------------------------------------- 64-point register DFT
// W64^k, k < 48, fp32-rounded from fp64 (the products b*c of dft64 stay below 46)
__device__ constexpr float kW64[48][2] = {
    {1.000000000e+00f, 0.000000000e+00f},
    {9.951847196e-01f, -9.801714122e-02f},
    {9.807852507e-01f, -1.950903237e-01f},
    {9.569403529e-01f, -2.902846634e-01f},
    {9.238795042e-01f, -3.826834261e-01f},
    {8.819212914e-01f, -4.713967443e-01f},
    {8.314695954e-01f, -5.555702448e-01f},
    {7.730104327e-01f, -6.343932748e-01f},
    {7.071067691e-01f, -7.071067691e-01f},
    {6.343932748e-01f, -7.730104327e-01f},
    {5.555702448e-01f, -8.314695954e-01f},
    {4.713967443e-01f, -8.819212914e-01f},
    {3.826834261e-01f, -9.238795042e-01f},
    {2.902846634e-01f, -9.569403529e-01f},
    {1.950903237e-01f, -9.807852507e-01f},
    {9.801714122e-02f, -9.951847196e-01f},
    {6.123234263e-17f, -1.000000000e+00f},
    {-9.801714122e-02f, -9.951847196e-01f},
    {-1.950903237e-01f, -9.807852507e-01f},
    {-2.902846634e-01f, -9.569403529e-01f},
    {-3.826834261e-01f, -9.238795042e-01f},
    {-4.713967443e-01f, -8.819212914e-01f},
    {-5.555702448e-01f, -8.314695954e-01f},
    {-6.343932748e-01f, -7.730104327e-01f},
    {-7.071067691e-01f, -7.071067691e-01f},
    {-7.730104327e-01f, -6.343932748e-01f},
    {-8.314695954e-01f, -5.555702448e-01f},
    {-8.819212914e-01f, -4.713967443e-01f},
    {-9.238795042e-01f, -3.826834261e-01f},
    {-9.569403529e-01f, -2.902846634e-01f},
    {-9.807852507e-01f, -1.950903237e-01f},
    {-9.951847196e-01f, -9.801714122e-02f},
    {-1.000000000e+00f, -1.224646853e-16f},
    {-9.951847196e-01f, 9.801714122e-02f},
    {-9.807852507e-01f, 1.950903237e-01f},
    {-9.569403529e-01f, 2.902846634e-01f},
    {-9.238795042e-01f, 3.826834261e-01f},
    {-8.819212914e-01f, 4.713967443e-01f},
    {-8.314695954e-01f, 5.555702448e-01f},
    {-7.730104327e-01f, 6.343932748e-01f},
    {-7.071067691e-01f, 7.071067691e-01f},
    {-6.343932748e-01f, 7.730104327e-01f},
    {-5.555702448e-01f, 8.314695954e-01f},
    {-4.713967443e-01f, 8.819212914e-01f},
    {-3.826834261e-01f, 9.238795042e-01f},
    {-2.902846634e-01f, 9.569403529e-01f},
    {-1.950903237e-01f, 9.807852507e-01f},
    {-9.801714122e-02f, 9.951847196e-01f}

};

// In-place natural-order DFT of 64 registers: n = 16a + b, k = c + 4d,
//   X[c + 4d] = sum_b W16^{bd} [ W64^{bc} sum_a x[16a + b] W4^{ac} ]
// -- 16 DFT4 (stride 16), 45 constant twiddles, 4 DFT16 (contiguous), a register rename.
__device__ __forceinline__ void dft64(float2 (&v)[64]) {
#pragma unroll
    for (int b = 0; b < 16; ++b) dft4(v[b], v[16 + b], v[32 + b], v[48 + b]);
#pragma unroll
    for (int c = 1; c < 4; ++c) {
#pragma unroll
        for (int b = 1; b < 16; ++b) {
            const int e = b * c;
            if (e == 16) v[b + 16 * c] = cmul_mj(v[b + 16 * c]);
            else v[b + 16 * c] = cmul(v[b + 16 * c], make_float2(kW64[e][0], kW64[e][1]));
        }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) dft16(&v[16 * c]);
    float2 x[64];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int d = 0; d < 16; ++d) x[c + 4 * d] = v[16 * c + d];
#pragma unroll
    for (int k = 0; k < 64; ++k) v[k] = x[k];
}


}  // namespace rsp
