// rsp_capi.cpp -- the C ABI (include/rsp.h): context, parameter validation, fp64 host
// precomputation (matched-filter spectra, twiddle tables, windows), device buffer pools
// and the chunked PC -> MTD(+Doppler CFAR) -> range CFAR pipeline.
//
// Chunking: the pulse-compression output of `chunk` CPIs is written to a scratch buffer
// that is read back by the MTD kernel right after; chunk * P * R_out * 8 bytes is sized
// (default 64 MiB) to stay in the 256 MiB Infinity Cache, so the corner turn between
// the fast-time (PC) and slow-time (MTD) passes is served on-die instead of from HBM.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <complex>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <exception>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rsp.h"
#include "rsp_hostpool.h"
#include "rsp_internal.h"

using cd = std::complex<double>;

struct DevBuf {
    void* p = nullptr;
    size_t n = 0;
};

struct rsp_ctx {
    int device = 0;
    bool cfar_only = false;   // created with params == NULL
    rsp_params p{};
    std::string err;
    hipStream_t stream = nullptr;
    rsp::PcArgs pc{};
    bool pc_v2 = false;                 // per-segment specialised kernels (pc_mf_kernel)
#ifndef RSP_PC_OLS_MIN
// 4096: an 8192-point segment (c4) runs as 3 blocks of 4096 points at four workgroups per CU
// instead of one whole-row transform at two: PC 289-301 -> 275-282 us per c4 step, chain +1.2-2.3 %
// (profiles/r04/ab/session9_ols4k.txt; dev-only -D for A/B of the threshold)
#define RSP_PC_OLS_MIN 4096
#endif
    int pc_ols_min = RSP_PC_OLS_MIN;    // overlap-save split of segments longer than this
    std::vector<rsp::PcMfArgs> pc_mf_whole, pc_mf_split;   // per MF segment, for rsp_set_pc_split
    std::vector<rsp::PcMfArgs> pc_mf;   // one launch per matched-filter segment
    rsp::MtdArgs mtd{};
    int64_t V = 0;                      // Doppler rows (rsp_params.mtd_nfft or P)
    int beams = 1;                      // 2: DMX left/right pair
    size_t pc_lds = 0;
    int64_t chunk = 0;  // 0 = default
    int nstreams = 0;   // chunk pipelines (the caller's stream + nstreams-1 internal ones); 0 = default
    hipStream_t aux[3] = {nullptr, nullptr, nullptr};
    hipEvent_t ev_fork = nullptr, ev_join[3] = {nullptr, nullptr, nullptr};
    // The context's scratch (PC corner turn, hit lists, internal RDM, flagV staging) is reused by
    // every _dev call: a call's stream waits for the previous call's release event first, so
    // calls on different streams never overlap on it.
    hipEvent_t ev_scratch = nullptr;
    bool scratch_pending = false;
    std::vector<void*> owned;           // constant tables (freed at destroy)
    std::map<int, float2*> tw;          // twiddle tables by length
    DevBuf scratch_pc, tmp_flagV, tmp_rdm;
    // range concatenation between PC and MTD (rsp_set_range_concat, fun_lss_range_concate):
    // PC rows are pc_w wide (the params' R_out); the MTD and every output see p.R_out = the sum
    // of the ncat parts; cat_tmp holds the full-width PC rows of each pipeline
    int64_t pc_w = 0;
    int ncat = 0;
    int64_t cat_src[RSP_MAX_SEG] = {}, cat_len[RSP_MAX_SEG] = {};
    DevBuf cat_tmp;
    DevBuf pf_gain;                     // fused iSTC gains (rsp_set_prefilter)
    DevBuf hit_list;                    // per-lane Doppler-hit lists (fused range CFAR)
    DevBuf hit_ctr;                     // per-lane, per-MTD-workgroup hit counts
    DevBuf meas_band;                   // measurement: per-(CPI, band, column) hit counts
    DevBuf ing_meta;                    // ingest: per-PRT record offsets and types
    DevBuf st_in, st_canon, st_rdm, st_flag, st_flagV, st_t;  // host-API staging (rsp_cfar)
    // Pipelined host-buffer path (rsp_pc_mtd_cfar / rsp_pc_mtd): chunk k's H2D (copy stream),
    // chain (ctx->stream) and D2H (copy stream) overlap chunks k+1 and k-1; pageable <-> pinned
    // staging through rings of pinned pieces, copied by a host thread pool.
    struct HostPipe {
        static constexpr int kSlots = 2;      // chunk slots (device buffers)
        static constexpr int kRing = 4;       // pinned pieces per direction
        hipStream_t s_h2d = nullptr, s_d2h = nullptr;
        DevBuf in[kSlots], canon[kSlots], rdm[kSlots], flag[kSlots], flagV[kSlots], tr[kSlots][3];
        hipEvent_t ev_in[kSlots] = {}, ev_comp[kSlots] = {}, ev_out[kSlots] = {};
        void* pin_in[kRing] = {};
        void* pin_out[kRing] = {};
        hipEvent_t ev_pin_in[kRing] = {}, ev_pin_out[kRing] = {};
        size_t piece = 0;                     // bytes per pinned piece
        int ring_in = 0;                      // next input piece slot
        int threads = 0;                      // requested copy threads (0 = default)
        std::unique_ptr<rsp::CopyPool> pool;
        std::unique_ptr<rsp::Prefaulter> prefault;   // fresh output arrays (host_prefault)
        rsp::Prefaulter* pf = nullptr;                // the running call's prefault job, if any
        // one-chunk calls (host_chain_small): pinned staging the kernels read and write directly
        static constexpr int kParts = 16;     // output parts in flight (one event each)
        void* zc_in = nullptr;
        void* zc_out = nullptr;
        size_t zc_in_n = 0, zc_out_n = 0;
        hipEvent_t ev_part[kParts] = {};
    } hp;
    int64_t host_chunk = 0;                   // CPIs per host chunk (0 = by bytes)
    // diagnostics (rsp_profile): HIP event pairs around each kernel launch
    struct Ev {
        int k;
        hipEvent_t a, b;
    };
    int prof = 0;            // 0 off; N >= 1: bracket every N-th launch
    uint64_t prof_tick = 0;
    std::vector<Ev> evs;
    size_t nev = 0;
    double prof_ms[RSP_NKERNELS] = {};
    int64_t prof_n[RSP_NKERNELS] = {};
};

static thread_local std::string g_err;

static int fail(rsp_ctx* ctx, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (ctx) ctx->err = buf;
    g_err = buf;
    return code;
}

#define HIP_TRY(ctx, expr)                                                                   \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return fail((ctx), RSP_ERR_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_),   \
                        __FILE__, __LINE__);                                                 \
    } while (0)

// ------------------------------------------------------------------ host numerics (fp64)
static double mround(double x) { return x >= 0 ? std::floor(x + 0.5) : -std::floor(-x + 0.5); }

static double bessel_i0(double x) {
    double sum = 1.0, term = 1.0, q = x * x / 4.0;
    for (int k = 1; k < 500; ++k) {
        term *= q / ((double)k * k);
        sum += term;
        if (term < 1e-18 * sum) break;
    }
    return sum;
}

static std::vector<double> make_window(int kind, double beta, int64_t n) {
    std::vector<double> w((size_t)n, 1.0);
    if (n == 1) return w;
    for (int64_t k = 0; k < n; ++k) {
        if (kind == RSP_WIN_KAISER) {
            double r = ((double)k - (n - 1) / 2.0) / ((n - 1) / 2.0);
            double a = 1.0 - r * r;
            w[k] = bessel_i0(beta * std::sqrt(a > 0 ? a : 0.0)) / bessel_i0(beta);
        } else if (kind == RSP_WIN_HAMMING) {
            w[k] = 0.54 - 0.46 * std::cos(2.0 * M_PI * (double)k / (double)(n - 1));
        }
    }
    return w;
}

// in-place radix-2 forward FFT, n a power of two
static void fft_pow2(std::vector<cd>& a) {
    const size_t n = a.size();
    for (size_t i = 1, j = 0; i < n; ++i) {
        size_t bit = n >> 1;
        for (; j & bit; bit >>= 1) j ^= bit;
        j ^= bit;
        if (i < j) std::swap(a[i], a[j]);
    }
    for (size_t len = 2; len <= n; len <<= 1) {
        for (size_t i = 0; i < n; i += len) {
            for (size_t k = 0; k < len / 2; ++k) {
                const double ang = -2.0 * M_PI * (double)k / (double)len;
                const cd w(std::cos(ang), std::sin(ang));
                const cd u = a[i + k], v = a[i + k + len / 2] * w;
                a[i + k] = u + v;
                a[i + k + len / 2] = u - v;
            }
        }
    }
}

template <typename T>
static int upload(rsp_ctx* ctx, const std::vector<T>& h, T** out) {
    void* d = nullptr;
    HIP_TRY(ctx, hipMalloc(&d, h.size() * sizeof(T)));
    ctx->owned.push_back(d);
    HIP_TRY(ctx, hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    *out = (T*)d;
    return RSP_OK;
}

static int twiddles(rsp_ctx* ctx, int n, const float2** out) {
    auto it = ctx->tw.find(n);
    if (it != ctx->tw.end()) {
        *out = it->second;
        return RSP_OK;
    }
    std::vector<float2> h((size_t)n);
    for (int e = 0; e < n; ++e) {
        const double ang = -2.0 * M_PI * (double)e / (double)n;
        h[e] = make_float2((float)std::cos(ang), (float)std::sin(ang));
    }
    float2* d = nullptr;
    int rc = upload(ctx, h, &d);
    if (rc) return rc;
    ctx->tw[n] = d;
    *out = d;
    return RSP_OK;
}

// H = conj(FFT_n(scale * replica)) / n in fp64 (fft(x, n) truncates), and the n-point twiddles
static int mf_spectrum(rsp_ctx* ctx, const rsp_pc_segment& g, int n, const float2** H, const float2** tw) {
    std::vector<cd> a((size_t)n, cd(0, 0));
    const int64_t L = g.coef_len < n ? g.coef_len : n;
    for (int64_t k = 0; k < L; ++k) a[k] = g.scale * cd(g.coef_re[k], g.coef_im ? g.coef_im[k] : 0.0);
    fft_pow2(a);
    std::vector<float2> h((size_t)n);
    for (int64_t k = 0; k < n; ++k) {
        const cd v = std::conj(a[k]) / (double)n;
        h[k] = make_float2((float)v.real(), (float)v.imag());
    }
    float2* dh = nullptr;
    int rc = upload(ctx, h, &dh);
    if (rc) return rc;
    *H = dh;
    return twiddles(ctx, n, tw);
}

// Overlap-save split of a long matched-filter segment (fun_lss_pulse_compression.m:64-72:
// ifft(fft(x, nfft) .* conj(fft(h, nfft)))).  With nfft >= out_len + hlen - 1 no output of the
// nfft-point circular correlation wraps, so output n = sum_k x[n + k] conj(h[k]) (x zero past
// in_len) -- the same sums as nsub blocks of an nb-point correlation, block j producing outputs
// [j*step, (j+1)*step), step = nb - hlen + 1.  A 16384-point row needs one 139 KB LDS slot
// (one workgroup per CU, every phase exposed); nb = 4096 blocks run four workgroups per CU.
// Kept only where it is exact in that sense and the FIR does not ride on the segment.
static int pc_overlap_save(rsp_ctx* ctx, const rsp_pc_segment& g, rsp::PcMfArgs& a) {
    a.nsub = 0;
    a.sub_step = 0;
    const int64_t nfft = a.mf.nfft;
    const int64_t hlen = g.coef_len < nfft ? g.coef_len : nfft;
    if (nfft <= ctx->pc_ols_min || a.do_fir || nfft < (int64_t)a.mf.out_len + hlen - 1) return RSP_OK;
    int best = 0, best_n = 0, best_step = 0;
    for (int nb : {8192, 4096, 2048}) {   // (ties: the longer block, fewer re-read samples)
        if (nb >= nfft) continue;
        const int64_t step = nb - hlen + 1;
        if (step < nb / 2) continue;
        const int64_t n = (a.mf.out_len + step - 1) / step;
        if (!best || n * nb < (int64_t)best_n * best) {
            best = nb;
            best_n = (int)n;
            best_step = (int)step;
        }
    }
    if (!best || (int64_t)best_n * best >= 2 * nfft) return RSP_OK;
    int rc = mf_spectrum(ctx, g, best, &a.mf.H, &a.mf.tw);
    if (rc) return rc;
    a.mf.nfft = best;
    a.nsub = best_n;
    a.sub_step = best_step;
    return RSP_OK;
}

static int ensure(rsp_ctx* ctx, DevBuf& b, size_t bytes) {
    if (b.n >= bytes && b.p) return RSP_OK;
    if (b.p) {
        HIP_TRY(ctx, hipFree(b.p));
        b.p = nullptr;
        b.n = 0;
    }
    if (bytes == 0) return RSP_OK;
    HIP_TRY(ctx, hipMalloc(&b.p, bytes));
    b.n = bytes;
    return RSP_OK;
}

static void zero_v_band(int64_t rows, int div, int* lo, int* hi) {
    if (div <= 0) {
        *lo = 0;
        *hi = 0;
        return;
    }
    const int64_t zv = (int64_t)mround(rows / 2.0);
    const int64_t k = (int64_t)mround((double)rows / (double)div);
    int64_t a = zv - k - 1, b = zv + k;
    if (a < 0) a = 0;
    if (b > rows) b = rows;
    *lo = (int)a;
    *hi = (int)(b > a ? b : a);
}

// ------------------------------------------------------------------ public API
const char* rsp_version(void) { return "rsp-mi355x 0.5.0 (gfx950, abi 4)"; }

const char* rsp_last_error(const rsp_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

int rsp_destroy(rsp_ctx* ctx) {
    if (!ctx) return RSP_OK;
    hipSetDevice(ctx->device);
    for (void* p : ctx->owned) hipFree(p);
    DevBuf* bufs[] = {&ctx->pf_gain, &ctx->scratch_pc, &ctx->cat_tmp, &ctx->tmp_flagV, &ctx->tmp_rdm, &ctx->hit_list, &ctx->hit_ctr,
                      &ctx->st_in, &ctx->st_canon, &ctx->st_rdm, &ctx->st_flag, &ctx->st_flagV, &ctx->st_t,
                      &ctx->meas_band, &ctx->ing_meta};
    for (DevBuf* b : bufs)
        if (b->p) hipFree(b->p);
    for (auto& e : ctx->evs) {
        hipEventDestroy(e.a);
        hipEventDestroy(e.b);
    }
    for (int i = 0; i < 3; ++i) {
        if (ctx->aux[i]) hipStreamDestroy(ctx->aux[i]);
        if (ctx->ev_join[i]) hipEventDestroy(ctx->ev_join[i]);
    }
    {
        auto& h = ctx->hp;
        for (int i = 0; i < h.kSlots; ++i) {
            DevBuf* hb[] = {&h.in[i], &h.canon[i], &h.rdm[i], &h.flag[i], &h.flagV[i], &h.tr[i][0], &h.tr[i][1],
                            &h.tr[i][2]};
            for (DevBuf* b : hb)
                if (b->p) hipFree(b->p);
            if (h.ev_in[i]) hipEventDestroy(h.ev_in[i]);
            if (h.ev_comp[i]) hipEventDestroy(h.ev_comp[i]);
            if (h.ev_out[i]) hipEventDestroy(h.ev_out[i]);
        }
        if (h.zc_in) hipHostFree(h.zc_in);
        if (h.zc_out) hipHostFree(h.zc_out);
        for (auto& e : h.ev_part)
            if (e) hipEventDestroy(e);
        for (int i = 0; i < h.kRing; ++i) {
            if (h.pin_in[i]) hipHostFree(h.pin_in[i]);
            if (h.pin_out[i]) hipHostFree(h.pin_out[i]);
            if (h.ev_pin_in[i]) hipEventDestroy(h.ev_pin_in[i]);
            if (h.ev_pin_out[i]) hipEventDestroy(h.ev_pin_out[i]);
        }
        if (h.s_h2d) hipStreamDestroy(h.s_h2d);
        if (h.s_d2h) hipStreamDestroy(h.s_d2h);
        h.pool.reset();
    }
    if (ctx->ev_fork) hipEventDestroy(ctx->ev_fork);
    if (ctx->ev_scratch) hipEventDestroy(ctx->ev_scratch);
    if (ctx->stream) hipStreamDestroy(ctx->stream);
    delete ctx;
    return RSP_OK;
}

int rsp_create(rsp_ctx** out, int device, const rsp_params* prm) {
    if (!out) return fail(nullptr, RSP_ERR_ARG, "rsp_create: null argument");
    *out = nullptr;
    if (!prm) {   // CFAR-only context (rsp_cfar / rsp_cfar_dev): a device and a stream
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
            return fail(nullptr, RSP_ERR_HIP, "rsp_create: no HIP device available");
        if (device < 0 || device >= ndev)
            return fail(nullptr, RSP_ERR_ARG, "rsp_create: device %d out of range (%d devices)", device, ndev);
        rsp_ctx* ctx = new rsp_ctx();
        ctx->device = device;
        ctx->cfar_only = true;
        if (hipSetDevice(device) != hipSuccess ||
            hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
            delete ctx;
            return fail(nullptr, RSP_ERR_HIP, "rsp_create: device/stream setup failed");
        }
        *out = ctx;
        return RSP_OK;
    }
    const rsp_params& p = *prm;
    if (p.P < 2 || p.R < 1 || p.R_out < 1 || p.R > (1 << 24) || p.R_out > (1 << 24))
        return fail(nullptr, RSP_ERR_SHAPE, "rsp_create: bad P=%lld R=%lld R_out=%lld",
                    (long long)p.P, (long long)p.R, (long long)p.R_out);
    const int64_t V = p.mtd_nfft ? p.mtd_nfft : p.P;
    const int beams = p.beams ? p.beams : 1;
    if (beams < 1 || beams > 2) return fail(nullptr, RSP_ERR_ARG, "rsp_create: beams=%d (1 or 2)", p.beams);
    if (V < p.P)
        return fail(nullptr, RSP_ERR_SHAPE, "rsp_create: mtd_nfft=%lld < P=%lld", (long long)V, (long long)p.P);
    const bool bluestein = !rsp::mtd_size_supported((int)V, beams) && beams == 1 && V == p.P &&
                           rsp::mtd_bluestein_nf((int)V) > 0;
    if (!rsp::mtd_size_supported((int)V, beams) && !bluestein)
        return fail(nullptr, RSP_ERR_UNSUPPORTED,
                    "rsp_create: Doppler length %lld (beams %d) not built (radix plans 2^k, 3*2^k up to 2048; "
                    "other even and odd P <= 1024 by Bluestein; two beams: 512, 1024, 2048)",
                    (long long)V, beams);
    if (p.zero_ends < 0 || 2 * (int64_t)p.zero_ends > V)
        return fail(nullptr, RSP_ERR_ARG, "rsp_create: zero_ends=%d out of range", p.zero_ends);
    if (p.nseg < 0 || p.nseg > RSP_MAX_SEG)
        return fail(nullptr, RSP_ERR_ARG, "rsp_create: nseg=%d out of range", p.nseg);
    if (p.window < RSP_WIN_KAISER || p.window > RSP_WIN_RECT)
        return fail(nullptr, RSP_ERR_ARG, "rsp_create: bad window %d", p.window);

    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(nullptr, RSP_ERR_HIP, "rsp_create: no HIP device available");
    if (device < 0 || device >= ndev)
        return fail(nullptr, RSP_ERR_ARG, "rsp_create: device %d out of range (%d devices)", device, ndev);

    rsp_ctx* ctx = new rsp_ctx();
    ctx->device = device;
    ctx->p = p;
    ctx->pc_w = p.R_out;
    for (int s = 0; s < RSP_MAX_SEG; ++s) ctx->p.seg[s].coef_re = ctx->p.seg[s].coef_im = nullptr;
    auto bail = [&](int rc) {
        g_err = ctx->err;
        rsp_destroy(ctx);
        return rc;
    };
    if (hipSetDevice(device) != hipSuccess) return bail(fail(ctx, RSP_ERR_HIP, "hipSetDevice(%d) failed", device));
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess)
        return bail(fail(ctx, RSP_ERR_HIP, "hipStreamCreate failed"));

    // ---- pulse-compression segments
    rsp::PcArgs& pc = ctx->pc;
    pc.P = (int)p.P;
    pc.R = (int)p.R;
    pc.R_out = (int)p.R_out;
    pc.nseg = p.nseg;
    std::vector<char> covered((size_t)p.R_out, 0);
    int max_nfft = 64;
    for (int s = 0; s < p.nseg; ++s) {
        const rsp_pc_segment& g = p.seg[s];
        rsp::SegDev& d = pc.seg[s];
        std::memset(&d, 0, sizeof(d));
        if (g.in_start < 0 || g.in_len < 1 || g.in_start + g.in_len > p.R)
            return bail(fail(ctx, RSP_ERR_ARG, "segment %d: input [%lld,+%lld) outside R=%lld", s,
                             (long long)g.in_start, (long long)g.in_len, (long long)p.R));
        if (g.out_start < 0 || g.out_len < 1 || g.out_start + g.out_len > p.R_out)
            return bail(fail(ctx, RSP_ERR_ARG, "segment %d: output [%lld,+%lld) outside R_out=%lld", s,
                             (long long)g.out_start, (long long)g.out_len, (long long)p.R_out));
        for (int64_t c = g.out_start; c < g.out_start + g.out_len; ++c) {
            if (covered[c]) return bail(fail(ctx, RSP_ERR_ARG, "segment %d overlaps another segment's output", s));
            covered[c] = 1;
        }
        if (!g.coef_re || g.coef_len < 1)
            return bail(fail(ctx, RSP_ERR_ARG, "segment %d: missing coefficients", s));
        d.kind = g.kind;
        d.in_start = (int)g.in_start;
        d.in_len = (int)g.in_len;
        d.out_start = (int)g.out_start;
        d.out_len = (int)g.out_len;
        d.scale = (float)g.scale;
        if (g.kind == RSP_SEG_FIR) {
            if (g.coef_len > RSP_MAX_FIR_TAPS)
                return bail(fail(ctx, RSP_ERR_UNSUPPORTED, "segment %d: %lld FIR taps > %d", s,
                                 (long long)g.coef_len, RSP_MAX_FIR_TAPS));
            if (g.out_len != g.in_len)
                return bail(fail(ctx, RSP_ERR_ARG, "segment %d: FIR needs out_len == in_len", s));
            d.ntaps = (int)g.coef_len;
            std::vector<float> tf((size_t)d.ntaps);
            for (int k = 0; k < d.ntaps; ++k) d.taps[k] = tf[k] = (float)g.coef_re[k];
            float* dt = nullptr;
            int rc = upload(ctx, tf, &dt);
            if (rc) return bail(rc);
            d.taps_dev = dt;
            d.ntaps4 = (d.ntaps + 3) & ~3;
            std::vector<float2> t2((size_t)d.ntaps4, float2{0.f, 0.f});
            for (int k = 0; k < d.ntaps; ++k) {
                const float b = (float)(g.coef_re[k] * g.scale);
                t2[k] = float2{b, b};
            }
            float2* dt2 = nullptr;
            rc = upload(ctx, t2, &dt2);
            if (rc) return bail(rc);
            d.taps2_dev = dt2;
            int64_t sh = g.fir_shift % g.out_len;
            if (sh < 0) sh += g.out_len;
            d.fir_shift = (int)sh;
        } else if (g.kind == RSP_SEG_MF) {
            if (!rsp::pc_nfft_supported((int)g.nfft))
                return bail(fail(ctx, RSP_ERR_UNSUPPORTED, "segment %d: nfft=%lld not built (2^k, 64..16384)", s,
                                 (long long)g.nfft));
            if (g.in_len > g.nfft || g.out_len > g.nfft)
                return bail(fail(ctx, RSP_ERR_ARG, "segment %d: in_len/out_len exceed nfft", s));
            d.nfft = (int)g.nfft;
            if (d.nfft > max_nfft) max_nfft = d.nfft;
            int rc = mf_spectrum(ctx, g, d.nfft, &d.H, &d.tw);
            if (rc) return bail(rc);
        } else {
            return bail(fail(ctx, RSP_ERR_ARG, "segment %d: bad kind %d", s, g.kind));
        }
    }
    // output columns no segment writes stay 0 (s_PC_0 = zeros, fun_lss_pulse_compression.m:27)
    pc.nzero = 0;
    for (int64_t c = 0; c < p.R_out;) {
        if (covered[c]) { ++c; continue; }
        int64_t e = c;
        while (e < p.R_out && !covered[e]) ++e;
        if (pc.nzero >= RSP_MAX_SEG + 1)
            return bail(fail(ctx, RSP_ERR_UNSUPPORTED, "too many uncovered output column ranges"));
        pc.zero_lo[pc.nzero] = (int)c;
        pc.zero_hi[pc.nzero] = (int)e;
        ++pc.nzero;
        c = e;
    }
    ctx->pc_lds = rsp::pc_lds_bytes(max_nfft);
    // Specialised path: at most one FIR segment, every MF length built, FIR staged in a slot
    {
        int nfir = 0, nmf = 0, fir_idx = -1;
        bool ok = true;
        for (int s = 0; s < p.nseg; ++s) {
            if (pc.seg[s].kind == RSP_SEG_FIR) { ++nfir; fir_idx = s; }
            else ++nmf;
        }
        ok = nfir <= 1 && nmf >= 1;
        int first = 1;
        for (int s = 0; s < p.nseg && ok; ++s) {
            if (pc.seg[s].kind != RSP_SEG_MF) continue;
            rsp::PcMfArgs a;
            std::memset(&a, 0, sizeof(a));
            a.R = (int)p.R;
            a.R_out = (int)p.R_out;
            a.mf = pc.seg[s];
            if (first) {
                a.do_fir = fir_idx >= 0;
                if (a.do_fir) a.fir = pc.seg[fir_idx];
                a.nzero = pc.nzero;
                for (int z = 0; z < pc.nzero; ++z) {
                    a.zero_lo[z] = pc.zero_lo[z];
                    a.zero_hi[z] = pc.zero_hi[z];
                }
                if (!rsp::pc_mf_supported(a.mf.nfft, a.do_fir ? rsp::fir_stage_len(a.fir) : 0)) ok = false;
                first = 0;
            } else if (!rsp::pc_mf_supported(a.mf.nfft, 0)) {
                ok = false;
            }
            ctx->pc_mf_whole.push_back(a);
            if (ok) {
                const int rc = pc_overlap_save(ctx, p.seg[s], a);
                if (rc) return bail(rc);
            }
            ctx->pc_mf_split.push_back(a);
            ctx->pc_mf.push_back(a);
        }
        ctx->pc_v2 = ok;
        if (!ok) {
            ctx->pc_mf.clear();
            ctx->pc_mf_whole.clear();
            ctx->pc_mf_split.clear();
        }
    }

    // ---- MTD
    rsp::MtdArgs& m = ctx->mtd;
    ctx->V = V;
    ctx->beams = beams;
    m.P = (int)V;            // Doppler FFT length; pulses beyond pin are the zero padding
    m.pin = (int)p.P;
    m.beams = beams;
    m.R_out = (int)p.R_out;
    m.shift = p.fftshift ? (int)(V / 2) : 0;
    if (p.zero_ends > 0) {   // rows [V-n+1, V) and [0, n): a band wrapping through row 0
        m.z_lo = (int)(V - p.zero_ends + 1);
        m.z_hi = (int)(V + p.zero_ends);
    } else {
        zero_v_band(V, p.zero_v_div, &m.z_lo, &m.z_hi);
    }
    std::vector<double> w = make_window(p.window, p.window_beta, p.P);   // window(P), zero-padded
    std::vector<float> wf((size_t)V, 0.f);
    for (int64_t i = 0; i < p.P; ++i) wf[(size_t)i] = (float)w[(size_t)i];
    float* dw = nullptr;
    int rc = upload(ctx, wf, &dw);
    if (rc) return bail(rc);
    m.win = dw;
    if (bluestein) {
        // X[k] = c[k] sum_n (x[n] w[n] c[n]) conj(c[k-n]), c[n] = exp(-j pi n^2 / V): tables in
        // fp64 (n^2 reduced mod 2V so the phase stays exact), the chirp spectrum by FFT
        const int nf = rsp::mtd_bluestein_nf((int)V);
        auto chirp = [&](int64_t n) {
            const double ph = -M_PI * (double)((n * n) % (2 * V)) / (double)V;
            return cd(std::cos(ph), std::sin(ph));
        };
        std::vector<float2> bwc((size_t)nf, float2{0.f, 0.f}), bsp((size_t)nf);
        for (int64_t n = 0; n < V; ++n) {
            const cd z = w[(size_t)n] * chirp(n);
            bwc[(size_t)n] = float2{(float)z.real(), (float)z.imag()};
        }
        std::vector<cd> b((size_t)nf, cd(0, 0));
        for (int64_t n = 0; n < V; ++n) {
            b[(size_t)n] = std::conj(chirp(n));
            if (n) b[(size_t)(nf - n)] = std::conj(chirp(n));
        }
        fft_pow2(b);
        for (int i = 0; i < nf; ++i) bsp[(size_t)i] = float2{(float)(b[(size_t)i].real() / nf), (float)(b[(size_t)i].imag() / nf)};
        float2 *dbwc = nullptr, *dbsp = nullptr;
        if ((rc = upload(ctx, bwc, &dbwc))) return bail(rc);
        if ((rc = upload(ctx, bsp, &dbsp))) return bail(rc);
        m.bnf = nf;
        m.bwc = dbwc;
        m.bspec = dbsp;
        rc = twiddles(ctx, nf, &m.tw);
    } else {
        rc = twiddles(ctx, (int)V, &m.tw);
    }
    if (rc) return bail(rc);
    *out = ctx;
    return RSP_OK;
}

// MTD/fun_lss_pulse_compression.m:31 (also DMX_SignalProcessing_main_xzr.m:146)
static const double kFirTaps[35] = {-9, -7, -2, 10, 27, 40, 42, 24, -13, -57, -89, -86, -30, 77, 220, 364, 471, 511,
                                    471, 364, 220, 77, -30, -86, -89, -57, -13, 24, 42, 40, 27, 10, -2, -7, -9};

static int64_t colon_count(double a, double d, double b) {   // MATLAB a:d:b length
    const double q = (b - a) / d;
    const double r = std::floor(q + 0.5);
    return (std::fabs(q - r) < 1e-9 * (std::fabs(q) > 1 ? std::fabs(q) : 1.0) ? (int64_t)r : (int64_t)std::floor(q)) + 1;
}

static int64_t nextpow2(int64_t n) {
    int64_t p = 64;
    while (p < n) p <<= 1;
    return p;
}

int rsp_create_v2(rsp_ctx** out, int device, int64_t P, int64_t R, const int64_t point_prt[4], double fs,
                  double B, const double tao[3]) {
    if (!out || !point_prt || !tao || fs <= 0 || tao[1] <= 0 || tao[2] <= 0)
        return fail(nullptr, RSP_ERR_ARG, "rsp_create_v2: bad argument");
    const int64_t p1 = point_prt[1], p2 = point_prt[2], p3 = point_prt[3];
    if (p1 < 1 || p2 < 1 || p3 < 1 || p1 + p2 + p3 > R)
        return fail(nullptr, RSP_ERR_SHAPE, "rsp_create_v2: point_prt segments exceed R=%lld", (long long)R);
    const double ts = 1.0 / fs;
    std::vector<double> re[2], im[2];
    for (int k = 0; k < 2; ++k) {   // pulse2 (K = -B/tau2), pulse3 (K = +B/tau3): fun_MTD_produce.m:62-69
        const double tau = tao[k + 1], K = (k == 0 ? -B : B) / tau;
        const int64_t n = colon_count(-tau / 2, ts, tau / 2 - ts);
        re[k].resize((size_t)n);
        im[k].resize((size_t)n);
        for (int64_t i = 0; i < n; ++i) {
            const double t = -tau / 2 + ts * (double)i;
            const double ph = 2.0 * M_PI * 0.5 * K * t * t;
            re[k][i] = std::cos(ph);
            im[k][i] = std::sin(ph);
        }
    }
    std::vector<double> taps(35);
    for (int i = 0; i < 35; ++i) taps[i] = kFirTaps[i] / 511.0;   // filter_coef / max (:32)
    rsp_params prm;
    std::memset(&prm, 0, sizeof(prm));
    prm.P = P;
    prm.R = R;
    prm.R_out = R;
    prm.nseg = 3;
    prm.window = RSP_WIN_KAISER;
    prm.window_beta = 8.0;
    prm.fftshift = 1;
    prm.zero_v_div = 150;
    rsp_pc_segment& a = prm.seg[0];
    a.kind = RSP_SEG_FIR;
    a.fir_shift = 17;   // round(mean(grpdelay(b))) of the symmetric 35-tap FIR (:47)
    a.in_start = 0;
    a.in_len = a.out_len = p1;
    a.scale = 1.0 / 1.2;
    a.coef_len = 35;
    a.coef_re = taps.data();
    const int64_t m3 = R - p1 - p2;
    for (int k = 0; k < 2; ++k) {
        rsp_pc_segment& g = prm.seg[k + 1];
        g.kind = RSP_SEG_MF;
        g.in_start = g.out_start = k == 0 ? p1 : p1 + p2;
        g.in_len = k == 0 ? p2 : m3;
        g.out_len = k == 0 ? p2 : p3;
        g.coef_len = (int64_t)re[k].size();
        g.nfft = nextpow2(g.in_len + g.coef_len - 1);
        g.scale = 1.0;
        g.coef_re = re[k].data();
        g.coef_im = im[k].data();
    }
    return rsp_create(out, device, &prm);
}

int rsp_create_legacy(rsp_ctx** out, int device, int64_t P, int64_t R, const double* pulse2_re,
                      const double* pulse2_im, int64_t n2, const double* pulse3_re, const double* pulse3_im,
                      int64_t n3) {
    if (!out || !pulse2_re || !pulse2_im || !pulse3_re || !pulse3_im || n2 < 1 || n3 < 1)
        return fail(nullptr, RSP_ERR_ARG, "rsp_create_legacy: bad argument");
    const int64_t p1 = 82, p2 = 242, p3 = R - 324;   // fun_MTD_produce.m:24-38 (legacy)
    if (p3 < 1) return fail(nullptr, RSP_ERR_SHAPE, "rsp_create_legacy: R=%lld <= 324", (long long)R);
    std::vector<double> taps(35);
    for (int i = 0; i < 35; ++i) taps[i] = kFirTaps[i] / 511.0;   // filter_coef / max
    rsp_params prm;
    std::memset(&prm, 0, sizeof(prm));
    prm.P = P;
    prm.R = R;
    prm.R_out = R;
    prm.nseg = 3;
    prm.window = RSP_WIN_KAISER;
    prm.window_beta = 8.0;
    prm.fftshift = 1;
    prm.zero_v_div = 150;
    rsp_pc_segment& a = prm.seg[0];
    a.kind = RSP_SEG_FIR;
    a.fir_shift = 0;    // the legacy version keeps the FIR's group delay
    a.in_start = 0;
    a.in_len = a.out_len = p1;
    a.scale = 1.0 / 1.2;
    a.coef_len = 35;
    a.coef_re = taps.data();
    const double* re[2] = {pulse2_re, pulse3_re};
    const double* im[2] = {pulse2_im, pulse3_im};
    const int64_t n[2] = {n2, n3};
    const int64_t m3 = R - p1 - p2;
    for (int k = 0; k < 2; ++k) {
        rsp_pc_segment& g = prm.seg[k + 1];
        g.kind = RSP_SEG_MF;
        g.in_start = g.out_start = k == 0 ? p1 : p1 + p2;
        g.in_len = k == 0 ? p2 : m3;
        g.out_len = k == 0 ? p2 : p3;
        g.coef_len = n[k];
        g.nfft = nextpow2(g.in_len + g.coef_len - 1);
        g.scale = 1.0;
        g.coef_re = re[k];
        g.coef_im = im[k];
    }
    return rsp_create(out, device, &prm);
}

int rsp_set_streams(rsp_ctx* ctx, int32_t n) {
    if (!ctx) return fail(nullptr, RSP_ERR_ARG, "rsp_set_streams: null ctx");
    if (n < 0 || n > 4) return fail(ctx, RSP_ERR_ARG, "rsp_set_streams: n must be 0..4");
    ctx->nstreams = n;   // 0: the mode-dependent default
    return RSP_OK;
}

int rsp_set_chunk(rsp_ctx* ctx, int64_t cpis) {
    if (!ctx) return fail(nullptr, RSP_ERR_ARG, "rsp_set_chunk: null ctx");
    if (cpis < 0) return fail(ctx, RSP_ERR_ARG, "rsp_set_chunk: negative chunk");
    ctx->chunk = cpis;
    return RSP_OK;
}


static bool set_device(rsp_ctx* ctx) { return hipSetDevice(ctx->device) == hipSuccess; }

static int64_t chunk_of(const rsp_ctx* ctx, int64_t batch) {
    int64_t c = ctx->chunk;
    if (c <= 0) {
        const int64_t per = (ctx->V > ctx->beams * ctx->p.P ? ctx->V : ctx->beams * ctx->p.P) * ctx->p.R_out * 8;
        c = (64ll << 20) / (per > 0 ? per : 1);
        if (c < 1) c = 1;
    }
    if (c > batch) c = batch;
    if (c > 65535) c = 65535;
    return c;
}

// CFAR argument blocks from the public struct; validates like MATLAB would fail.
static int build_cfar(rsp_ctx* ctx, const rsp_cfar_params* cf, int64_t V, int64_t R,
                      rsp::CfarVArgs* cv, rsp::CfarRArgs* cr) {
    if (cf->refV < 1 || cf->saveV < 0 || cf->refR < 1 || cf->saveR < 0)
        return fail(ctx, RSP_ERR_ARG, "CFAR: reference cells must be >= 1 and guard cells >= 0");
    if (cf->M0 < 0 || 2 * (int64_t)cf->M0 + 1 > V)
        return fail(ctx, RSP_ERR_ARG, "CFAR: M0=%d leaves no rows of %lld", cf->M0, (long long)V);
    if (cf->nseg < 0 || cf->nseg > RSP_MAX_SEG) return fail(ctx, RSP_ERR_ARG, "CFAR: bad nseg %d", cf->nseg);
    const int lo = cf->M0 + 1, hi = (int)V - cf->M0;
    if (hi - lo < 2 * (cf->saveV + cf->refV))
        return fail(ctx, RSP_ERR_CFAR_WINDOW,
                    "CFAR: %d Doppler cells after stripping M0 rows < 2*(guard+ref)=%d "
                    "(Function_CFAR1D_sub would index out of range)",
                    hi - lo, 2 * (cf->saveV + cf->refV));
    int nseg = cf->nseg;
    int64_t slo[RSP_MAX_SEG], shi[RSP_MAX_SEG];
    if (nseg == 0) {
        nseg = 1;
        slo[0] = 0;
        shi[0] = R;
    } else {
        for (int s = 0; s < nseg; ++s) {
            slo[s] = cf->seg_lo[s];
            shi[s] = cf->seg_hi[s];
            if (slo[s] < 0 || shi[s] > R || shi[s] <= slo[s])
                return fail(ctx, RSP_ERR_ARG, "CFAR: segment %d [%lld,%lld) outside [0,%lld)", s,
                            (long long)slo[s], (long long)shi[s], (long long)R);
            for (int q = 0; q < s; ++q)
                if (slo[s] < shi[q] && slo[q] < shi[s]) return fail(ctx, RSP_ERR_ARG, "CFAR: segments overlap");
        }
    }
    if (cf->rFlag && cf->saveR + cf->refR + 2 > 32)
        return fail(ctx, RSP_ERR_UNSUPPORTED, "CFAR: range guard+ref = %d > 30 not built", cf->saveR + cf->refR);
    if (cf->rFlag)
        for (int s = 0; s < nseg; ++s)
            if (shi[s] - slo[s] < 2 * (cf->saveR + cf->refR))
                return fail(ctx, RSP_ERR_CFAR_WINDOW,
                            "CFAR: range segment %d has %lld cells < 2*(guard+ref)=%d", s,
                            (long long)(shi[s] - slo[s]), 2 * (cf->saveR + cf->refR));
    int cz_lo, cz_hi;
    zero_v_band(V, cf->zero_v_div, &cz_lo, &cz_hi);
    std::memset(cv, 0, sizeof(*cv));
    cv->enabled = 1;
    cv->lo = lo;
    cv->hi = hi;
    cv->ref = cf->refV;
    cv->save = cf->saveV;
    cv->method = cf->methodV;
    cv->T = (float)cf->TV;
    cv->Tr = (float)(cf->TV / cf->refV);
    cv->cz_lo = cz_lo;
    cv->cz_hi = cz_hi;
    cv->nseg = nseg;
    std::memset(cr, 0, sizeof(*cr));
    cr->V = (int)V;
    cr->R = (int)R;
    cr->lo = lo;
    cr->hi = hi;
    cr->rflag = cf->rFlag ? 1 : 0;
    cr->ref = cf->refR;
    cr->save = cf->saveR;
    cr->method = cf->methodR;
    cr->T = (float)cf->TR;
    cr->Tr = (float)(cf->TR / cf->refR);
    cr->cz_lo = cz_lo;
    cr->cz_hi = cz_hi;
    cr->nseg = nseg;
    for (int s = 0; s < nseg; ++s) {
        cv->seg_lo[s] = cr->seg_lo[s] = (int)slo[s];
        cv->seg_hi[s] = cr->seg_hi[s] = (int)shi[s];
    }
    return RSP_OK;
}


// Order this call's use of the context scratch after the previous call's (on any stream).
static int scratch_acquire(rsp_ctx* ctx, hipStream_t s) {
    if (ctx->scratch_pending) HIP_TRY(ctx, hipStreamWaitEvent(s, ctx->ev_scratch, 0));
    return RSP_OK;
}
static int scratch_release(rsp_ctx* ctx, hipStream_t s) {
    if (!ctx->ev_scratch) HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->ev_scratch, hipEventDisableTiming));
    HIP_TRY(ctx, hipEventRecord(ctx->ev_scratch, s));
    ctx->scratch_pending = true;
    return RSP_OK;
}

static hipError_t run_pc(rsp_ctx* ctx, const void* ein, int dtype, float2* out, int64_t rows, hipStream_t s,
                         int slot = 0);

// Run one kernel launch, bracketed by HIP events on `s` when profiling is on (every
// ctx->prof-th launch: a timing event costs the stream a few microseconds, so a sampled
// bracket keeps the measured region's throughput unchanged).
template <typename F>
static hipError_t timed(rsp_ctx* ctx, int k, hipStream_t s, F&& launch) {
    if (!ctx->prof) return launch();
    if (ctx->prof_tick++ % (uint64_t)ctx->prof != 0) return launch();
    if (ctx->nev == ctx->evs.size()) {
        rsp_ctx::Ev e{k, nullptr, nullptr};
        hipError_t r = hipEventCreate(&e.a);
        if (r == hipSuccess) r = hipEventCreate(&e.b);
        if (r != hipSuccess) return r;
        ctx->evs.push_back(e);
    }
    rsp_ctx::Ev& e = ctx->evs[ctx->nev++];
    e.k = k;
    hipError_t r = hipEventRecord(e.a, s);
    if (r != hipSuccess) return r;
    r = launch();
    if (r != hipSuccess) return r;
    return hipEventRecord(e.b, s);
}

static hipError_t run_pc_rows(rsp_ctx* ctx, const void* ein, int dtype, float2* out, int64_t rows, hipStream_t s);
// Pulse compression of `rows` echo rows into `out` ([rows][R_out]).  With a range concatenation
// (rsp_set_range_concat) the full-width PC rows land in cat_tmp slot `slot` (ensured by the caller:
// slot * rows * pc_w complex per slot) and the parts are gathered into `out` by 2-D copies on s.
static hipError_t run_pc(rsp_ctx* ctx, const void* ein, int dtype, float2* out, int64_t rows, hipStream_t s,
                         int slot) {
    if (ctx->ncat == 0) return run_pc_rows(ctx, ein, dtype, out, rows, s);
    float2* full = (float2*)ctx->cat_tmp.p + (size_t)slot * rows * ctx->pc_w;
    hipError_t e = run_pc_rows(ctx, ein, dtype, full, rows, s);
    if (e != hipSuccess) return e;
    const size_t so = sizeof(float2);
    int64_t dst = 0;
    for (int i = 0; i < ctx->ncat; ++i) {
        e = hipMemcpy2DAsync(out + dst, (size_t)ctx->p.R_out * so, full + ctx->cat_src[i], (size_t)ctx->pc_w * so,
                             (size_t)ctx->cat_len[i] * so, (size_t)rows, hipMemcpyDeviceToDevice, s);
        if (e != hipSuccess) return e;
        dst += ctx->cat_len[i];
    }
    return hipSuccess;
}
static int cat_ensure(rsp_ctx* ctx, int slots, int64_t rows) {
    return ctx->ncat ? ensure(ctx, ctx->cat_tmp, (size_t)slots * rows * ctx->pc_w * sizeof(float2)) : RSP_OK;
}

int rsp_set_range_concat(rsp_ctx* ctx, int32_t nparts, const int64_t* src_start, const int64_t* len) {
    if (!ctx) return fail(nullptr, RSP_ERR_ARG, "rsp_set_range_concat: null ctx");
    if (ctx->cfar_only) return fail(ctx, RSP_ERR_ARG, "rsp_set_range_concat: CFAR-only context");
    if (nparts < 0 || nparts > RSP_MAX_SEG || (nparts > 0 && (!src_start || !len)))
        return fail(ctx, RSP_ERR_ARG, "rsp_set_range_concat: bad part list (%d parts)", nparts);
    int64_t w = 0;
    for (int i = 0; i < nparts; ++i) {
        if (len[i] < 1 || src_start[i] < 0 || src_start[i] + len[i] > ctx->pc_w)
            return fail(ctx, RSP_ERR_ARG, "rsp_set_range_concat: part %d [%lld, +%lld) outside the %lld PC columns", i,
                        (long long)src_start[i], (long long)len[i], (long long)ctx->pc_w);
        w += len[i];
    }
    if (!set_device(ctx)) return fail(ctx, RSP_ERR_HIP, "hipSetDevice failed");
    HIP_TRY(ctx, hipDeviceSynchronize());   // no launch in flight still uses the old width
    ctx->ncat = nparts;
    for (int i = 0; i < nparts; ++i) {
        ctx->cat_src[i] = src_start[i];
        ctx->cat_len[i] = len[i];
    }
    ctx->p.R_out = nparts > 0 ? w : ctx->pc_w;
    ctx->mtd.R_out = (int)ctx->p.R_out;
    return RSP_OK;
}

static hipError_t run_pc_rows(rsp_ctx* ctx, const void* ein, int dtype, float2* out, int64_t rows, hipStream_t s) {
    if (!ctx->pc_v2)
        return timed(ctx, RSP_K_PC, s, [&] { return rsp::launch_pc(ein, dtype, out, rows, ctx->pc, ctx->pc_lds, s); });
    if (ctx->pc_mf.size() == 2 && rsp::pc_pair_supported(ctx->pc_mf[0].mf.nfft, ctx->pc_mf[1].mf.nfft)) {
        rsp::PcMfArgs a1 = ctx->pc_mf[0], a2 = ctx->pc_mf[1];
        a1.rows = a2.rows = (int)rows;
        return timed(ctx, RSP_K_PC, s, [&] { return rsp::launch_pc_mf(ein, dtype, out, a1, &a2, s); });
    }
    for (const rsp::PcMfArgs& a0 : ctx->pc_mf) {
        rsp::PcMfArgs a = a0;
        a.rows = (int)rows;
        hipError_t e = timed(ctx, RSP_K_PC, s, [&] { return rsp::launch_pc_mf(ein, dtype, out, a, nullptr, s); });
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

int rsp_profile(rsp_ctx* ctx, int32_t enable) {
    if (!ctx) return fail(nullptr, RSP_ERR_ARG, "rsp_profile: null ctx");
    if (enable < 0) return fail(ctx, RSP_ERR_ARG, "rsp_profile: enable %d < 0", enable);
    ctx->prof = enable;
    ctx->prof_tick = 0;
    ctx->nev = 0;
    for (int k = 0; k < RSP_NKERNELS; ++k) {
        ctx->prof_ms[k] = 0;
        ctx->prof_n[k] = 0;
    }
    return RSP_OK;
}

int rsp_profile_read_n(rsp_ctx* ctx, double* ms, int64_t* launches, int32_t n) {
    if (!ctx || !ms || !launches || n < 0) return fail(ctx, RSP_ERR_ARG, "rsp_profile_read_n: bad argument");
    for (size_t i = 0; i < ctx->nev; ++i) {
        rsp_ctx::Ev& e = ctx->evs[i];
        HIP_TRY(ctx, hipEventSynchronize(e.b));
        float t = 0.f;
        HIP_TRY(ctx, hipEventElapsedTime(&t, e.a, e.b));
        ctx->prof_ms[e.k] += t;
        ctx->prof_n[e.k] += 1;
    }
    ctx->nev = 0;
    for (int k = 0; k < n && k < RSP_NKERNELS; ++k) {
        ms[k] = ctx->prof_ms[k];
        launches[k] = ctx->prof_n[k];
    }
    return RSP_OK;
}

// the ABI-3 form: exactly the four kernel ids that header declared (RSP_K_PC .. RSP_K_CFAR_V)
int rsp_profile_read(rsp_ctx* ctx, double* ms, int64_t* launches) {
    if (!ctx || !ms || !launches) return fail(ctx, RSP_ERR_ARG, "rsp_profile_read: null argument");
    return rsp_profile_read_n(ctx, ms, launches, 4);
}

int rsp_pc_dev(rsp_ctx* ctx, const void* d_echo, int32_t dtype, int64_t batch, void* d_pc, void* stream) {
    if (!ctx || !d_echo || !d_pc || batch < 0) return fail(ctx, RSP_ERR_ARG, "rsp_pc_dev: bad argument");
    if (ctx->cfar_only) return fail(ctx, RSP_ERR_ARG, "context was created for CFAR only (params == NULL)");
    if (dtype != RSP_C64 && dtype != RSP_C32F16) return fail(ctx, RSP_ERR_ARG, "rsp_pc_dev: dtype %d", dtype);
    if (!set_device(ctx)) return fail(ctx, RSP_ERR_HIP, "hipSetDevice failed");
    if (ctx->ncat == 0) {
        HIP_TRY(ctx, run_pc(ctx, d_echo, dtype, (float2*)d_pc, batch * ctx->p.P, (hipStream_t)stream));
        return RSP_OK;
    }
    // the concatenation stages full-width rows in the context's scratch
    hipStream_t s = (hipStream_t)stream;
    int rc = scratch_acquire(ctx, s);
    if (rc) return rc;
    if ((rc = cat_ensure(ctx, 1, batch * ctx->p.P))) return rc;
    HIP_TRY(ctx, run_pc(ctx, d_echo, dtype, (float2*)d_pc, batch * ctx->p.P, s));
    return scratch_release(ctx, s);
}

int rsp_set_pc_split(rsp_ctx* ctx, int32_t enable) {
    if (!ctx) return fail(nullptr, RSP_ERR_ARG, "rsp_set_pc_split: null ctx");
    if (ctx->cfar_only) return fail(ctx, RSP_ERR_ARG, "rsp_set_pc_split: CFAR-only context");
    if (!ctx->pc_v2)   // the generic PC path has no split to select
        return fail(ctx, RSP_ERR_UNSUPPORTED, "rsp_set_pc_split: this context has no specialised PC path");
    const std::vector<rsp::PcMfArgs>& src = enable ? ctx->pc_mf_split : ctx->pc_mf_whole;
    for (size_t i = 0; i < ctx->pc_mf.size() && i < src.size(); ++i) {
        const float* gain = ctx->pc_mf[i].gain;   // the fused pre-filter stays as set
        ctx->pc_mf[i] = src[i];
        ctx->pc_mf[i].gain = gain;
    }
    return RSP_OK;
}

int rsp_set_prefilter(rsp_ctx* ctx, const float* gain, int32_t mti_lag) {
    if (!ctx) return fail(nullptr, RSP_ERR_ARG, "rsp_set_prefilter: null ctx");
    if (ctx->cfar_only) return fail(ctx, RSP_ERR_ARG, "rsp_set_prefilter: CFAR-only context");
    if (mti_lag < 0) return fail(ctx, RSP_ERR_ARG, "rsp_set_prefilter: negative MTI lag %d", mti_lag);
    if (gain && !ctx->pc_v2)
        return fail(ctx, RSP_ERR_UNSUPPORTED, "rsp_set_prefilter: the fused gain needs the per-segment PC kernels");
    if (!set_device(ctx)) return fail(ctx, RSP_ERR_HIP, "hipSetDevice failed");
    HIP_TRY(ctx, hipDeviceSynchronize());   // no launch in flight still reads the old gains
    const float* d_gain = nullptr;
    if (gain) {
        const size_t bytes = (size_t)ctx->p.R * sizeof(float);
        const int rc = ensure(ctx, ctx->pf_gain, bytes);
        if (rc) return rc;
        HIP_TRY(ctx, hipMemcpy(ctx->pf_gain.p, gain, bytes, hipMemcpyHostToDevice));
        d_gain = (const float*)ctx->pf_gain.p;
    }
    for (rsp::PcMfArgs& a : ctx->pc_mf) a.gain = d_gain;
    ctx->mtd.mti_lag = mti_lag;
    return RSP_OK;
}

// The chain over `units` on stream s.  win == 0: a unit is one CPI ([P][R] input rows).
// win > 0: a unit is a frame pair (n, n+1) of a frame-contiguous input holding units + 1
// frames, producing `win` windowed CPIs (MtdArgs::win); a chunk computes the PC of its
// frames plus the look-ahead frame once, and every window reads its rows from that PC.
// Where a chunk's range stage (executeCFAR's range test of the Doppler hits) runs:
//   2 (default): grouped -- the range stages of up to kRangeGroup consecutive chunks of a lane run
//     as one launch behind the group's last MTD; the MTD records hit indices relative to the
//     group's first output cell (MtdArgs::cell_off).  Needs the caller's RDM (internal RDM slots
//     are reused) and a group span inside the range kernels' 2 GiB buffer window.
//   0: fused -- the stage rides in the next MTD launch on the lane (RangeJob57: gathers issued with
//     the tile loads); the fallback when grouping does not apply.
//   1: a standalone launch behind every chunk's MTD.
// Measured (profiles/r05/ab/range_stage_grouping.txt): the fused job costs the MTD ~10 % at c3
// even with 0.28 % hits; groups of 8-32 chunks: c3 +2 %, c5 +1.5-2.6 %, bit-identical; a launch
// per chunk: c3 -1 %.  Dev A/B: environment RSP_RANGE_MODE / RSP_RANGE_GROUP (read once).
static constexpr int kRangeGroup = 16;
static constexpr uint64_t kRangeGroupBytes = 1ull << 30;   // hit-list slots of one call's groups
static int range_mode() {
    static const int m = [] { const char* v = getenv("RSP_RANGE_MODE"); return v && *v ? atoi(v) : 2; }();
    return m;
}
static int range_group() {
    static const int g = [] { const char* v = getenv("RSP_RANGE_GROUP"); const int x = v && *v ? atoi(v) : kRangeGroup; return x < 1 ? 1 : x; }();
    return g;
}

static int run_chain_body(rsp_ctx* ctx, const void* d_echo, int32_t dtype, int64_t units, int win,
                          const rsp_cfar_params* cfar, float* d_rdm, uint8_t* d_flag, uint8_t* d_flagV,
                          float* d_diff, hipStream_t s, bool pc_input) {
    const int64_t P = ctx->p.P, R = ctx->p.R, Ro = ctx->p.R_out, V = ctx->V, NB = ctx->beams;
    const size_t esz = dtype == RSP_C64 ? 8 : 4;
    rsp::MtdArgs m = ctx->mtd;
    rsp::CfarRArgs cr{};
    if (cfar) {
        int rc = build_cfar(ctx, cfar, V, Ro, &m.cv, &cr);
        if (rc) return rc;
    } else {
        m.cv.enabled = 0;
    }
    const int64_t ocpi = win > 0 ? win : 1;               // output CPIs per unit
    m.nwin = win;
    for (int i = 0; i < win; ++i) m.win_start[i] = (int)mround((double)i * P / win);
    int64_t cu = chunk_of(ctx, units * ocpi);              // CPIs per chunk
    // Default pipelines: 2 (PC of one chunk overlaps MTD / CFAR of the other); window mode 1 with
    // chunks of >= 32 frame pairs (look-ahead PC overhead <= 1/32, fewer launch tails): c4 114.9k
    // windows/s against 111.9k at 16 pairs and 106.5k at 8 (round 3); two pipelines of 8 pairs
    // lost (2 x 144 MiB of scratch overflows the Infinity Cache)
    const int nsd = ctx->nstreams > 0 ? ctx->nstreams : (win > 0 ? 1 : 2);
    if (win > 0) {
        cu = cu / ocpi;
        if (ctx->chunk > 0) {
            cu = cu > 0 ? cu : 1;                          // explicit chunk (rsp_set_chunk): as asked
        } else if (cu < 32) {
            // at least 32 pairs, but never more cells per chunk slot than the 32-bit hit
            // indices address (down to the old minimum and below for the largest windows)
            const int64_t fit = (int64_t)(0xffffffffull / ((uint64_t)ocpi * (uint64_t)V * (uint64_t)Ro));
            cu = 32 < fit ? 32 : (fit > cu ? fit : cu);
            if (cu < 1) cu = 1;
        }
    }
    if (cu > units) cu = units;
    // Chunk boundaries: chunk k covers units [cstart[k], cstart[k + 1]), cu units each but the last.
    std::vector<int64_t> cstart{0};
    while (cstart.back() < units) cstart.push_back(cstart.back() + cu < units ? cstart.back() + cu : units);
    const int64_t nchunks = (int64_t)cstart.size() - 1;
    const int ns = (int)(nsd < nchunks ? nsd : nchunks);
    const size_t plane = (size_t)V * Ro;                  // output cells per CPI
    const size_t cells = (size_t)cu * ocpi * plane;       // output cells per chunk slot
    const size_t pcrows = (size_t)(cu + (win > 0 ? 1 : 0)) * NB * P;
    int rc = pc_input ? RSP_OK : ensure(ctx, ctx->scratch_pc, (size_t)ns * pcrows * Ro * sizeof(float2));
    if (rc) return rc;
    if (!pc_input && (rc = cat_ensure(ctx, ns, (int64_t)pcrows))) return rc;
    int nreg = 0, reg = 0;
    if (cfar) {
        // fused range stage: per-lane hit lists, one region per MTD workgroup sized to its
        // cells (no overflow, no global atomics), and per-workgroup counts
        if (cells > 0xffffffffull) return fail(ctx, RSP_ERR_UNSUPPORTED, "chunk too large for 32-bit hit indices");
        // two slots per lane: chunk k's list is read by the next MTD launch on its lane while
        // that launch fills the other slot
        rsp::mtd_regions((int)V, (int)Ro, (int)(cu * ocpi), &nreg, &reg, (int)NB);
    }
    // grouped range stages (range_mode 2): a group's outputs must stay inside the range kernels'
    // 2 GiB buffer window, and the RDM must be the caller's (internal RDM slots are reused)
    int rgrp = range_group();
    if (cfar && nreg > 0) {   // the groups' hit-list slots within kRangeGroupBytes
        const uint64_t slot_bytes = (uint64_t)nreg * (uint64_t)reg * 4u;
        const uint64_t fit = kRangeGroupBytes / ((uint64_t)ns * slot_bytes);
        if ((uint64_t)rgrp > fit) rgrp = fit > 0 ? (int)fit : 1;
    }
    const bool grouped = cfar && cr.rflag && d_rdm && range_mode() == 2 && rgrp > 1 &&
                         ((uint64_t)(rgrp - 1) * (uint64_t)ns + 1u) * (uint64_t)cells * 4u < 0x80000000ull;   // (kOob, rsp_buf.h)
    // hit-list slots per lane: grouped, a group's range launch is stream-ordered before the next
    // group's first MTD on the lane, so the next group reuses the slots
    const int spl = grouped ? rgrp : 2;
    if (cfar) {
        rc = ensure(ctx, ctx->hit_list, (size_t)spl * ns * nreg * reg * sizeof(uint32_t));
        if (rc) return rc;
        rc = ensure(ctx, ctx->hit_ctr, (size_t)spl * ns * nreg * sizeof(uint32_t));
        if (rc) return rc;
    }
    if (!d_rdm) {   // internal RDM: two slots per lane for the same reason
        rc = ensure(ctx, ctx->tmp_rdm, (size_t)2 * ns * cells * sizeof(float));
        if (rc) return rc;
    }
    // the MTD kernels write the flag plane's zero background with the Doppler stage (every cell
    // of a CPI belongs to one MTD thread), and the range stage, stream-ordered after that
    // chunk's MTD launch, writes the 1s: no separate fill pass
    m.flag_zero = 1;
    // ... except for big chunks of long tiles: there a memset of the chunk's flag plane on the
    // lane before its MTD (a streaming fill) beats the tiles' 16-byte row-segment stores (tiles of
    // P >= 256 are 16 bins wide).  c4 (one 268 MB chunk per step): MTD 649 -> 572 us, +4.3 %;
    // c3 (32-bin tiles, 8 MiB chunks) -2.8 %, c5 (8 MiB chunks) neutral
    // (profiles/r05/ab/flag_memset.txt).  Dev A/B: RSP_FLAG_MEMSET 0 / 1 forces it off / on.
    static const int fenv = [] { const char* v = getenv("RSP_FLAG_MEMSET"); return v && *v ? atoi(v) : -1; }();
    const bool fm = cfar && cr.rflag && d_flag &&
                    (fenv >= 0 ? fenv == 1 : (V >= 256 && (uint64_t)cells >= (64ull << 20)));
    if (fm) m.flag_zero = 0;
    // (The fill on a side stream beside the chunk's PC, joined before the MTD, measured the same:
    // c4 133.8k vs 134.2k windows/s, three interleaved pairs, bit-identical -- the fill and the
    // PC share the HBM; profiles/r06/c4/flag_memset_side.txt.)
    // Chunk k runs on lane k % ns (lane 0 = the caller's stream), each lane with its own
    // scratch slot, so PC of one chunk overlaps MTD / CFAR of the previous one.  The lanes
    // fork from and join back into the caller's stream.
    hipStream_t lanes[4] = {s, nullptr, nullptr, nullptr};
    if (ns > 1) {
        if (!ctx->ev_fork) HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming));
        HIP_TRY(ctx, hipEventRecord(ctx->ev_fork, s));
        for (int i = 1; i < ns; ++i) {
            if (!ctx->aux[i - 1]) HIP_TRY(ctx, hipStreamCreateWithFlags(&ctx->aux[i - 1], hipStreamNonBlocking));
            if (!ctx->ev_join[i - 1]) HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->ev_join[i - 1], hipEventDisableTiming));
            lanes[i] = ctx->aux[i - 1];
            HIP_TRY(ctx, hipStreamWaitEvent(lanes[i], ctx->ev_fork, 0));
        }
    }
    // A chunk's range stage (its hit list) runs inside the next MTD launch on its lane, so the
    // lane timeline carries no separate small kernel; a lane's last chunk gets its own launch.
    struct Pending {
        int nreg = 0, reg = 0;
        const float* rdm = nullptr;
        uint8_t* flag = nullptr;
        const uint32_t* hits = nullptr;
        const uint32_t* counts = nullptr;
    } pend[4];
    for (int64_t k = 0; k < nchunks; ++k) {
        const int64_t u0 = cstart[(size_t)k];
        const int64_t n = cstart[(size_t)k + 1] - u0;
        const int64_t ncpi = n * ocpi;                     // CPIs this chunk produces
        const size_t o0 = (size_t)u0 * ocpi * plane;      // output offset
        const int lane = (int)(k % ns);
        const int64_t j = k / ns;                          // the chunk's index on its lane
        const int slot = lane * spl + (int)(j % spl);      // double-buffered per lane (grouped: one group)
        const int64_t jg0 = j - j % rgrp;                  // grouped: the group's first chunk on the lane
        const size_t og = grouped ? (size_t)cstart[(size_t)(lane + ns * jg0)] * ocpi * plane : o0;
        hipStream_t ls = lanes[lane];
        const char* ein = (const char*)d_echo + (size_t)u0 * NB * P * R * esz;
        float* rdm = d_rdm ? d_rdm + o0 : (float*)ctx->tmp_rdm.p + (lane * 2 + (int)(j & 1)) * cells;
        uint8_t* fv = (cfar && d_flagV) ? d_flagV + o0 : nullptr;
        float2* pcs;
        if (pc_input) {   // d_echo already holds pulse-compressed rows [units][beams][P][R_out]
            pcs = (float2*)d_echo + (size_t)u0 * NB * P * Ro;
        } else {
            pcs = (float2*)ctx->scratch_pc.p + lane * pcrows * Ro;
            HIP_TRY(ctx, run_pc(ctx, ein, dtype, pcs, (n + (win > 0 ? 1 : 0)) * NB * P, ls, lane));
        }
        m.diff = d_diff ? d_diff + o0 : nullptr;
        m.prev_nregions = 0;
        m.cell_off = (uint32_t)(o0 - og);   // hit indices relative to the group's first cell (else 0)
        if (cfar) {
            m.flag = d_flag + o0;
            m.rflag = cr.rflag;
            m.hits = (uint32_t*)ctx->hit_list.p + (size_t)slot * nreg * reg;
            m.hit_count = (uint32_t*)ctx->hit_ctr.p + (size_t)slot * nreg;
            const Pending& pv = pend[lane];
            if (pv.nreg > 0 && !grouped) {
                m.prev_rdm = pv.rdm;
                m.prev_flag = pv.flag;
                m.prev_hits = pv.hits;
                m.prev_count = pv.counts;
                m.prev_nregions = pv.nreg;
                m.prev_region = pv.reg;
                m.prev_cr = cr;
            }
        }
        if (fm) HIP_TRY(ctx, hipMemsetAsync(d_flag + o0, 0, (size_t)ncpi * plane, ls));
        HIP_TRY(ctx, timed(ctx, RSP_K_MTD, ls, [&] { return rsp::launch_mtd(pcs, rdm, fv, (int)ncpi, m, ls); }));
        if (cfar && cr.rflag) {
            Pending& pv = pend[lane];
            rsp::mtd_regions((int)V, (int)Ro, (int)ncpi, &pv.nreg, &pv.reg, (int)NB);   // this chunk's workgroups
            pv.rdm = rdm;
            pv.flag = m.flag;
            pv.hits = m.hits;
            pv.counts = m.hit_count;
            if (grouped) {   // the group's range stages, one launch behind its last MTD
                const bool last = k + ns >= nchunks;
                if (j % rgrp == rgrp - 1 || last) {
                    const int s0 = lane * spl + (int)(jg0 % spl);
                    const int nr = (int)(j - jg0) * nreg + pv.nreg;   // full chunks, then this one's regions
                    HIP_TRY(ctx, timed(ctx, RSP_K_CFAR_R, ls, [&] {
                        return rsp::launch_cfar_hits(d_rdm + og, d_flag + og, (uint32_t*)ctx->hit_list.p + (size_t)s0 * nreg * reg,
                                                     (uint32_t*)ctx->hit_ctr.p + (size_t)s0 * nreg, nr, pv.reg, cr, ls);
                    }));
                }
                pv.nreg = 0;
            } else if (range_mode() == 1) {   // (dev A/B) the chunk's range stage as its own launch, now
                HIP_TRY(ctx, timed(ctx, RSP_K_CFAR_R, ls, [&] {
                    return rsp::launch_cfar_hits(pv.rdm, pv.flag, pv.hits, pv.counts, pv.nreg, pv.reg, cr, ls);
                }));
                pv.nreg = 0;
            }
        }
    }
    for (int lane = 0; lane < ns; ++lane) {   // each lane's last chunk
        const Pending& pv = pend[lane];
        if (pv.nreg > 0)
            HIP_TRY(ctx, timed(ctx, RSP_K_CFAR_R, lanes[lane], [&] {
                return rsp::launch_cfar_hits(pv.rdm, pv.flag, pv.hits, pv.counts, pv.nreg, pv.reg, cr, lanes[lane]);
            }));
    }
    for (int i = 1; i < ns; ++i) {
        HIP_TRY(ctx, hipEventRecord(ctx->ev_join[i - 1], lanes[i]));
        HIP_TRY(ctx, hipStreamWaitEvent(s, ctx->ev_join[i - 1], 0));
    }
    return RSP_OK;
}

static int run_chain(rsp_ctx* ctx, const void* d_echo, int32_t dtype, int64_t units, int win,
                     const rsp_cfar_params* cfar, float* d_rdm, uint8_t* d_flag, uint8_t* d_flagV,
                     float* d_diff, hipStream_t s, bool pc_input = false) {
    int rc = scratch_acquire(ctx, s);
    if (rc) return rc;
    rc = run_chain_body(ctx, d_echo, dtype, units, win, cfar, d_rdm, d_flag, d_flagV, d_diff, s, pc_input);
    if (rc) return rc;
    return scratch_release(ctx, s);
}

static int check_chain_args(rsp_ctx* ctx, const char* fn, const void* d_echo, int32_t dtype, int64_t n,
                            const rsp_cfar_params* cfar, float* d_rdm, uint8_t* d_flag) {
    if (!ctx) return fail(nullptr, RSP_ERR_ARG, "%s: null ctx", fn);
    if (ctx->cfar_only) return fail(ctx, RSP_ERR_ARG, "context was created for CFAR only (params == NULL)");
    if (!d_echo || n < 0) return fail(ctx, RSP_ERR_ARG, "%s: bad input pointer/count", fn);
    if (dtype != RSP_C64 && dtype != RSP_C32F16)
        return fail(ctx, RSP_ERR_ARG, "%s: device dtype must be RSP_C64 or RSP_C32F16", fn);
    if (cfar && !d_flag) return fail(ctx, RSP_ERR_ARG, "%s: CFAR requested without d_flag", fn);
    if (!cfar && !d_rdm) return fail(ctx, RSP_ERR_ARG, "%s: no output requested", fn);
    return RSP_OK;
}

int rsp_pc_mtd_cfar_dev(rsp_ctx* ctx, const void* d_echo, int32_t dtype, int64_t batch,
                        const rsp_cfar_params* cfar, float* d_rdm, uint8_t* d_flag, uint8_t* d_flagV,
                        void* stream) {
    int rc = check_chain_args(ctx, "rsp_pc_mtd_cfar_dev", d_echo, dtype, batch, cfar, d_rdm, d_flag);
    if (rc) return rc;
    if (batch == 0) return RSP_OK;
    if (!set_device(ctx)) return fail(ctx, RSP_ERR_HIP, "hipSetDevice failed");
    return run_chain(ctx, d_echo, dtype, batch, 0, cfar, d_rdm, d_flag, d_flagV, nullptr, (hipStream_t)stream);
}

int rsp_mtd_cfar_dev(rsp_ctx* ctx, const void* d_pc, int64_t batch, const rsp_cfar_params* cfar, float* d_rdm,
                     uint8_t* d_flag, uint8_t* d_flagV, void* stream) {
    int rc = check_chain_args(ctx, "rsp_mtd_cfar_dev", d_pc, RSP_C64, batch, cfar, d_rdm, d_flag);
    if (rc) return rc;
    if (batch == 0) return RSP_OK;
    if (!set_device(ctx)) return fail(ctx, RSP_ERR_HIP, "hipSetDevice failed");
    return run_chain(ctx, d_pc, RSP_C64, batch, 0, cfar, d_rdm, d_flag, d_flagV, nullptr, (hipStream_t)stream, true);
}

int rsp_pc_mtd_cfar_diff_dev(rsp_ctx* ctx, const void* d_echo, int32_t dtype, int64_t batch,
                             const rsp_cfar_params* cfar, float* d_sum, float* d_diff, uint8_t* d_flag,
                             uint8_t* d_flagV, void* stream) {
    int rc = check_chain_args(ctx, "rsp_pc_mtd_cfar_diff_dev", d_echo, dtype, batch, cfar, d_sum, d_flag);
    if (rc) return rc;
    if (ctx->beams != 2)
        return fail(ctx, RSP_ERR_ARG, "rsp_pc_mtd_cfar_diff_dev: the context was created with beams=%d", ctx->beams);
    if (batch == 0) return RSP_OK;
    if (!set_device(ctx)) return fail(ctx, RSP_ERR_HIP, "hipSetDevice failed");
    return run_chain(ctx, d_echo, dtype, batch, 0, cfar, d_sum, d_flag, d_flagV, d_diff, (hipStream_t)stream);
}

int rsp_window_pc_mtd_cfar_dev(rsp_ctx* ctx, const void* d_frames, int32_t dtype, int64_t beams, int64_t frames,
                               int32_t win, const rsp_cfar_params* cfar, float* d_rdm, uint8_t* d_flag,
                               uint8_t* d_flagV, void* stream) {
    int rc = check_chain_args(ctx, "rsp_window_pc_mtd_cfar_dev", d_frames, dtype, frames, cfar, d_rdm, d_flag);
    if (rc) return rc;
    if (beams < 0) return fail(ctx, RSP_ERR_ARG, "rsp_window_pc_mtd_cfar_dev: beams %lld < 0", (long long)beams);
    if (ctx->beams != 1 || ctx->V != ctx->p.P)
        return fail(ctx, RSP_ERR_ARG, "rsp_window_pc_mtd_cfar_dev: needs a one-beam context with mtd_nfft = P");
    if (win < 1 || win > rsp::RSP_MAX_WIN)
        return fail(ctx, RSP_ERR_ARG, "rsp_window_pc_mtd_cfar_dev: win %d outside 1..%d", win, rsp::RSP_MAX_WIN);
    if (frames == 0 || beams == 0) return RSP_OK;
    if (!set_device(ctx)) return fail(ctx, RSP_ERR_HIP, "hipSetDevice failed");
    const int64_t P = ctx->p.P, R = ctx->p.R, Ro = ctx->p.R_out;
    const size_t esz = dtype == RSP_C64 ? 8 : 4;
    const size_t in_beam = (size_t)(frames + 1) * P * R * esz;    // bytes of one beam's frames
    const size_t out_beam = (size_t)frames * win * P * Ro;         // cells of one beam's windows
    for (int64_t b = 0; b < beams; ++b) {
        rc = run_chain(ctx, (const char*)d_frames + b * in_beam, dtype, frames, win, cfar,
                       d_rdm ? d_rdm + b * out_beam : nullptr, d_flag ? d_flag + b * out_beam : nullptr,
                       d_flagV ? d_flagV + b * out_beam : nullptr, nullptr, (hipStream_t)stream);
        if (rc) return rc;
    }
    return RSP_OK;
}

int rsp_cfar_dev(rsp_ctx* ctx, const float* d_rdm, int64_t V, int64_t R, int64_t batch,
                 const rsp_cfar_params* cfar, uint8_t* d_flag, uint8_t* d_flagV, void* stream) {
    if (!ctx) return fail(nullptr, RSP_ERR_ARG, "rsp_cfar_dev: null ctx");
    if (!d_rdm || !cfar || !d_flag || V < 1 || R < 1 || batch < 0)
        return fail(ctx, RSP_ERR_ARG, "rsp_cfar_dev: bad argument");
    if ((V + 1) * 4 > 64 * 1024 || R > (1 << 24))
        return fail(ctx, RSP_ERR_UNSUPPORTED, "rsp_cfar_dev: V=%lld or R=%lld too large", (long long)V, (long long)R);
    rsp::CfarVArgs cv;
    rsp::CfarRArgs cr;
    int rc = build_cfar(ctx, cfar, V, R, &cv, &cr);
    if (rc) return rc;
    if (!rsp::cfar_r_supported(cr))
        return fail(ctx, RSP_ERR_UNSUPPORTED,
                    "rsp_cfar_dev: a %lld-cell row with range window ref=%d guard=%d needs more than 160 KB of LDS "
                    "(only ref=5, guard=7 with R %% 4 == 0 is built for rows over 16320 cells)",
                    (long long)R, cr.ref, cr.save);
    if (batch == 0) return RSP_OK;
    if (!set_device(ctx)) return fail(ctx, RSP_ERR_HIP, "hipSetDevice failed");
    hipStream_t s = (hipStream_t)stream;
    const int64_t chunk = 65535;
    if ((rc = scratch_acquire(ctx, s))) return rc;
    if (!d_flagV) {
        rc = ensure(ctx, ctx->tmp_flagV, (size_t)(batch < chunk ? batch : chunk) * V * R);
        if (rc) return rc;
    }
    for (int64_t c0 = 0; c0 < batch; c0 += chunk) {
        const int64_t n = batch - c0 < chunk ? batch - c0 : chunk;
        const float* rdm = d_rdm + (size_t)c0 * V * R;
        uint8_t* fv = d_flagV ? d_flagV + (size_t)c0 * V * R : (uint8_t*)ctx->tmp_flagV.p;
        uint8_t* fl = d_flag + (size_t)c0 * V * R;
        HIP_TRY(ctx, timed(ctx, RSP_K_CFAR_V, s, [&] { return rsp::launch_cfar_v(rdm, fv, (int)n, (int)V, (int)R, cv, s); }));
        HIP_TRY(ctx, timed(ctx, RSP_K_CFAR_R, s, [&] { return rsp::launch_cfar_r(rdm, fv, fl, (int)n, cr, s); }));
    }
    return scratch_release(ctx, s);
}

// ------------------------------------------------------------------ post-detection measurement
int rsp_motion_measure_dev(rsp_ctx* ctx, const float* d_sum, const float* d_diff, const uint8_t* d_flag, int64_t V,
                           int64_t R, int64_t batch, const rsp_measure_params* mp, const double* d_r_scale,
                           const double* d_v_scale, int64_t max_hits, double* d_est, int32_t* d_cells,
                           int32_t* d_count, void* stream) {
    if (!ctx) return fail(nullptr, RSP_ERR_ARG, "rsp_motion_measure_dev: null ctx");
    if (!mp || !d_sum || !d_diff || !d_flag || !d_r_scale || !d_v_scale || !d_count || batch < 0 || max_hits < 0 ||
        (max_hits > 0 && !d_est))
        return fail(ctx, RSP_ERR_ARG, "rsp_motion_measure_dev: bad argument");
    const int64_t n = 2 * (int64_t)mp->extra_dots + 1;
    if (mp->extra_dots < 1 || mp->extra_dots > 4)
        return fail(ctx, RSP_ERR_UNSUPPORTED, "rsp_motion_measure_dev: extra_dots %d outside 1..4", mp->extra_dots);
    if (mp->r_interp < 1 || mp->r_interp > 64 || mp->v_interp < 1 || mp->v_interp > 64)
        return fail(ctx, RSP_ERR_ARG, "rsp_motion_measure_dev: interpolation factors %d, %d outside 1..64",
                    mp->r_interp, mp->v_interp);
    if (V < 1 || R < 1 || V > (1 << 20) || R > (1 << 20) || V * R > (int64_t)1 << 31 || batch > 0x7fffffff)
        return fail(ctx, RSP_ERR_ARG, "rsp_motion_measure_dev: bad shape %lld x %lld x %lld", (long long)batch,
                    (long long)V, (long long)R);
    if (R < n || mp->mtd0_num < 0 || V - 2 * (int64_t)mp->mtd0_num - 1 < n)
        return fail(ctx, RSP_ERR_ARG,
                    "rsp_motion_measure_dev: %lld range bins / %lld unzeroed rows are fewer than 2*extraDots+1",
                    (long long)R, (long long)(V - 2 * (int64_t)mp->mtd0_num - 1));
    const int64_t ld = mp->ld ? mp->ld : R, cs = mp->cpi_stride ? mp->cpi_stride : V * ld;
    if (ld < R || cs < (V - 1) * ld + R)
        return fail(ctx, RSP_ERR_ARG, "rsp_motion_measure_dev: row pitch %lld / CPI stride %lld too small for %lld x %lld",
                    (long long)ld, (long long)cs, (long long)V, (long long)R);
    if (batch == 0) return RSP_OK;
    if (!set_device(ctx)) return fail(ctx, RSP_ERR_HIP, "hipSetDevice failed");
    rsp::MeasureArgs a;
    a.ld = ld;
    a.cs = cs;
    a.extra_dots = mp->extra_dots;
    a.r_interp = mp->r_interp;
    a.v_interp = mp->v_interp;
    a.mtd0_num = mp->mtd0_num;
    a.beam_pos_num = mp->beam_pos_num;
    a.delta_r = mp->delta_r;
    a.delta_v = mp->delta_v;
    a.k_value = mp->k_value;
    a.beam_angle_step = mp->beam_angle_step;
    a.ele_comp = mp->ele_comp;
    a.ele_sys_err = mp->ele_sys_err;
    const int nb = rsp::measure_bands((int)V, (int)batch);
    int rc = scratch_acquire(ctx, (hipStream_t)stream);
    if (rc) return rc;
    if (nb > 1) {
        rc = ensure(ctx, ctx->meas_band, (size_t)batch * nb * R * sizeof(int32_t));
        if (rc != RSP_OK) return rc;
    }
    HIP_TRY(ctx, rsp::launch_measure(d_sum, d_diff, d_flag, (int)V, (int)R, (int)batch, a, d_r_scale, d_v_scale,
                                     max_hits, d_est, d_cells, d_count, (int32_t*)ctx->meas_band.p, nb,
                                     (hipStream_t)stream));
    return scratch_release(ctx, (hipStream_t)stream);
}

// ------------------------------------------------------------------ echo pre-filters
int rsp_prefilter_dev(rsp_ctx* ctx, const void* d_in, void* d_out, int64_t P, int64_t R, int64_t batch,
                      const float* d_gain, int32_t mti_lag, void* stream) {
    if (!ctx) return fail(nullptr, RSP_ERR_ARG, "rsp_prefilter_dev: null ctx");
    if (!d_in || !d_out || P < 1 || R < 2 || batch < 0 || mti_lag < 0)
        return fail(ctx, RSP_ERR_ARG, "rsp_prefilter_dev: bad argument");
    if (R % 2 != 0 || ((uintptr_t)d_in & 15) || ((uintptr_t)d_out & 15))
        return fail(ctx, RSP_ERR_UNSUPPORTED, "rsp_prefilter_dev: needs an even R and 16-byte aligned buffers");
    if (P > (1 << 24) || R > (1 << 24))
        return fail(ctx, RSP_ERR_ARG, "rsp_prefilter_dev: bad shape %lld x %lld", (long long)P, (long long)R);
    if (mti_lag > 0 && d_in == d_out)
        return fail(ctx, RSP_ERR_ARG, "rsp_prefilter_dev: MTI cannot run in place");
    if (batch == 0) return RSP_OK;
    if (!set_device(ctx)) return fail(ctx, RSP_ERR_HIP, "hipSetDevice failed");
    HIP_TRY(ctx, rsp::launch_prefilter((const float2*)d_in, (float2*)d_out, d_gain, (int)P, (int)R, batch, mti_lag,
                                       (hipStream_t)stream));
    return RSP_OK;
}

// ------------------------------------------------------------------ raw-data ingest
static int ingest_shape(rsp_ctx* ctx, const rsp_ingest_params* p, int64_t* rec) {
    if (!p) return fail(ctx, RSP_ERR_ARG, "ingest: null params");
    if (p->prt_num < 0 || p->point_prt <= 0 || p->channel_num <= 0 || p->channel_num > 255 || p->beam_num <= 0 ||
        p->bytes_head < 64 || p->bytes_realtime < 0 || p->bytes_tail < 0 || p->bytes_head % 4 || p->bytes_realtime % 4)
        return fail(ctx, RSP_ERR_ARG, "ingest: bad shape (prt %d, point %d, channels %d, beams %d, head %d)",
                    p->prt_num, p->point_prt, p->channel_num, p->beam_num, p->bytes_head);
    // FrameDataRead_xzr.m:108-119: DDC payload = samples * channels * 2 (I, Q) * 2 bytes, padded to 64 B
    int64_t sig = (int64_t)p->point_prt * p->channel_num * 4;
    if (sig % 64) sig += 64 - sig % 64;
    if (sig >= 0x80000000ll) return fail(ctx, RSP_ERR_UNSUPPORTED, "ingest: payload of %lld bytes", (long long)sig);
    *rec = (int64_t)p->bytes_head + p->bytes_realtime + sig + p->bytes_tail;
    return RSP_OK;
}

int rsp_ingest_record_bytes(const rsp_ingest_params* p, int64_t* bytes) {
    if (!bytes) return fail(nullptr, RSP_ERR_ARG, "rsp_ingest_record_bytes: null output");
    return ingest_shape(nullptr, p, bytes);
}

static int ingest_run(rsp_ctx* ctx, const char* who, bool ddc_only, const uint8_t* d_stream, int64_t nbytes,
                      const rsp_ingest_params* p, const float* d_dbf, void* d_out, int64_t beam_stride,
                      uint16_t* d_servo, int32_t* d_status, void* stream) {
    if (!ctx) return fail(nullptr, RSP_ERR_ARG, "%s: null ctx", who);
    int64_t rec = 0;
    int rc = ingest_shape(ctx, p, &rec);
    if (rc) return rc;
    if (!d_stream || nbytes < 0 || !d_dbf || !d_out || !d_status)
        return fail(ctx, RSP_ERR_ARG, "%s: null buffer or negative byte count", who);
    const int64_t plane = (int64_t)p->prt_num * p->point_prt;
    if (beam_stride == 0) beam_stride = plane;
    if (beam_stride < plane) return fail(ctx, RSP_ERR_ARG, "%s: beam_stride %lld < prt*point %lld", who,
                                         (long long)beam_stride, (long long)plane);
    if (p->prt_num == 0) return RSP_OK;
    if (!set_device(ctx)) return fail(ctx, RSP_ERR_HIP, "hipSetDevice failed");
    // per-PRT record offsets and types, written by the check kernel for the decode kernel
    // (stream-ordered on the caller's stream; one frame at a time per context)
    rc = ensure(ctx, ctx->ing_meta, (size_t)p->prt_num * (sizeof(int64_t) + sizeof(int32_t)));
    if (rc) return rc;
    rsp::IngestArgs a{};
    a.ddc_only = ddc_only ? 1 : 0;
    a.offs = (int64_t*)ctx->ing_meta.p;
    a.types = (int32_t*)((int64_t*)ctx->ing_meta.p + p->prt_num);
    a.prt_num = p->prt_num;
    a.point_prt = p->point_prt;
    a.channel_num = p->channel_num;
    a.beam_num = p->beam_num;
    a.bytes_head = p->bytes_head;
    a.bytes_realtime = p->bytes_realtime;
    a.bytes_tail = p->bytes_tail;
    a.rec_bytes = rec;
    a.beam_stride = beam_stride;
    HIP_TRY(ctx, rsp::launch_ingest(d_stream, nbytes, a, (const float2*)d_dbf, (float2*)d_out, d_servo, d_status,
                                    (hipStream_t)stream));
    return RSP_OK;
}

int rsp_ingest_ddc_dev(rsp_ctx* ctx, const uint8_t* d_stream, int64_t nbytes, const rsp_ingest_params* p,
                       const float* d_dbf, void* d_out, int64_t beam_stride, uint16_t* d_servo,
                       int32_t* d_status, void* stream) {
    return ingest_run(ctx, "rsp_ingest_ddc_dev", true, d_stream, nbytes, p, d_dbf, d_out, beam_stride, d_servo,
                      d_status, stream);
}

int rsp_ingest_frame_dev(rsp_ctx* ctx, const uint8_t* d_stream, int64_t nbytes, const rsp_ingest_params* p,
                         const float* d_dbf, void* d_out, int64_t beam_stride, uint16_t* d_servo,
                         int32_t* d_status, void* stream) {
    return ingest_run(ctx, "rsp_ingest_frame_dev", false, d_stream, nbytes, p, d_dbf, d_out, beam_stride, d_servo,
                      d_status, stream);
}

// ------------------------------------------------------------------ host-buffer entry points
static size_t dtype_size(int32_t dtype) {
    switch (dtype) {
        case RSP_C64: return 8;
        case RSP_C128: return 16;
        case RSP_C32F16: return 4;
        default: return 0;
    }
}

template <typename T>
static int fetch(rsp_ctx* ctx, const T* d, T* h, int64_t batch, int64_t A, int64_t B, int32_t layout) {
    const size_t n = (size_t)batch * A * B;
    if (layout == RSP_COLMAJOR) {
        int rc = ensure(ctx, ctx->st_t, n * sizeof(T));
        if (rc) return rc;
        hipError_t e;
        if (sizeof(T) == 4)
            e = rsp::launch_transpose_f32((const float*)d, (float*)ctx->st_t.p, batch, (int)A, (int)B, ctx->stream);
        else
            e = rsp::launch_transpose_u8((const uint8_t*)d, (uint8_t*)ctx->st_t.p, batch, (int)A, (int)B, ctx->stream);
        HIP_TRY(ctx, e);
        d = (const T*)ctx->st_t.p;
    }
    HIP_TRY(ctx, hipMemcpyAsync(h, d, n * sizeof(T), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return RSP_OK;
}

static int check_host_call(rsp_ctx* ctx, const void* echo, int32_t dtype, int32_t layout, int64_t P,
                           int64_t R, int64_t batch) {
    if (ctx->cfar_only) return fail(ctx, RSP_ERR_ARG, "context was created for CFAR only (params == NULL)");
    if (!echo || batch < 0) return fail(ctx, RSP_ERR_ARG, "null echo or negative batch");
    if (!dtype_size(dtype)) return fail(ctx, RSP_ERR_ARG, "bad dtype %d", dtype);
    if (layout != RSP_ROWMAJOR && layout != RSP_COLMAJOR) return fail(ctx, RSP_ERR_ARG, "bad layout %d", layout);
    if (P != ctx->p.P || R != ctx->p.R)
        return fail(ctx, RSP_ERR_SHAPE, "echo is %lld x %lld but the context was created for %lld x %lld",
                    (long long)P, (long long)R, (long long)ctx->p.P, (long long)ctx->p.R);
    if (!set_device(ctx)) return fail(ctx, RSP_ERR_HIP, "hipSetDevice failed");
    return RSP_OK;
}

// ---- pipelined host path
static constexpr size_t kHostPiece = 8u << 20;        // pinned piece
static constexpr size_t kHostChunkBytes = 32u << 20;  // device-side input bytes per host chunk
                                                      // (c3: 8 CPIs; tools/host_probe.py)

static int host_pipe_init(rsp_ctx* ctx) {
    auto& h = ctx->hp;
    if (h.s_h2d) return RSP_OK;
    HIP_TRY(ctx, hipStreamCreateWithFlags(&h.s_h2d, hipStreamNonBlocking));
    HIP_TRY(ctx, hipStreamCreateWithFlags(&h.s_d2h, hipStreamNonBlocking));
    for (int i = 0; i < h.kSlots; ++i) {
        HIP_TRY(ctx, hipEventCreateWithFlags(&h.ev_in[i], hipEventDisableTiming));
        HIP_TRY(ctx, hipEventCreateWithFlags(&h.ev_comp[i], hipEventDisableTiming));
        HIP_TRY(ctx, hipEventCreateWithFlags(&h.ev_out[i], hipEventDisableTiming));
    }
    for (auto& e : h.ev_part) HIP_TRY(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    h.piece = kHostPiece;
    for (int i = 0; i < h.kRing; ++i) {
        HIP_TRY(ctx, hipHostMalloc(&h.pin_in[i], h.piece, hipHostMallocDefault));
        HIP_TRY(ctx, hipHostMalloc(&h.pin_out[i], h.piece, hipHostMallocDefault));
        HIP_TRY(ctx, hipEventCreateWithFlags(&h.ev_pin_in[i], hipEventDisableTiming));
        HIP_TRY(ctx, hipEventCreateWithFlags(&h.ev_pin_out[i], hipEventDisableTiming));
    }
    return RSP_OK;
}

// (thread creation can throw: callers run inside rsp_pc_mtd_cfar's try block, which turns any
// exception into an error status -- nothing may unwind through the extern "C" boundary into
// the MEX host)
static rsp::CopyPool& host_pool(rsp_ctx* ctx) {
    auto& h = ctx->hp;
    int want = h.threads;
    if (want <= 0) {
        const unsigned hc = std::thread::hardware_concurrency();
        want = hc >= 16 ? 8 : (hc >= 4 ? (int)hc / 2 : 1);
    }
    if (!h.pool || h.pool->threads() != want) {
        h.pool.reset();
        h.pool.reset(new rsp::CopyPool(want));
    }
    return *h.pool;
}

// host (pageable) -> device, through the pinned input ring on the H2D stream: piece i is
// copied into a ring slot by the pool while the DMA of piece i-1 runs.
// Piece size for a transfer of `bytes`: the ring's 8 MiB, but at least four pieces per transfer
// down to 1 MiB, so a small call (one CPI: 8 MiB of C128 echo) still overlaps its memcpy with
// its DMA.
static size_t piece_for(const rsp_ctx* ctx, size_t bytes) {
    size_t p = (bytes / 4 + 4095) & ~(size_t)4095;
    if (p < ((size_t)1 << 20)) p = (size_t)1 << 20;
    return p < ctx->hp.piece ? p : ctx->hp.piece;
}

// `bytes` = the device-side bytes; narrow: src is complex double, narrowed to complex float on
// the way into the pinned piece (half the PCIe bytes of MATLAB's C128 echo).
// narrow 2: src is real double, narrowed to float the same way (rsp_cfar_f64).
static int h2d_pieces(rsp_ctx* ctx, void* d, const void* src, size_t bytes, int narrow = 0) {
    auto& h = ctx->hp;
    rsp::CopyPool& pool = host_pool(ctx);
    const size_t piece = piece_for(ctx, bytes);
    for (size_t off = 0; off < bytes; off += piece) {
        const size_t n = bytes - off < piece ? bytes - off : piece;
        const int r = h.ring_in;
        h.ring_in = (h.ring_in + 1) % h.kRing;
        HIP_TRY(ctx, hipEventSynchronize(h.ev_pin_in[r]));   // the slot's previous DMA is done
        if (narrow == 2)
            pool.narrow_f64((float*)h.pin_in[r], (const double*)((const char*)src + 2 * off), n / 4);
        else if (narrow)
            pool.narrow_c128((float*)h.pin_in[r], (const double*)((const char*)src + 2 * off), n / 8);
        else
            pool.copy(h.pin_in[r], (const char*)src + off, n);
        HIP_TRY(ctx, hipMemcpyAsync((char*)d + off, h.pin_in[r], n, hipMemcpyHostToDevice, h.s_h2d));
        HIP_TRY(ctx, hipEventRecord(h.ev_pin_in[r], h.s_h2d));
    }
    return RSP_OK;
}

// device -> host (pageable), through the pinned output ring on the D2H stream: up to kRing
// pieces in flight; each is copied out by the pool once its DMA is done.
// widen: the host side takes MATLAB's double -- 1: float cells, 2: 0/1 bytes -- converted by the
// pool as each pinned piece lands (bytes = device-side bytes; the host array is 8 bytes per element)
struct D2HPart {
    const void* d;
    void* h;
    size_t bytes;
    int widen = 0;
};
static int d2h_pieces(rsp_ctx* ctx, const std::vector<D2HPart>& parts) {
    auto& h = ctx->hp;
    rsp::CopyPool& pool = host_pool(ctx);
    struct Piece {
        const char* d;
        char* h;
        size_t n;
        int widen;
    };
    std::vector<Piece> ps;
    for (const D2HPart& p : parts) {
        const size_t piece = piece_for(ctx, p.bytes);
        const size_t scale = p.widen == 1 ? 2 : (p.widen == 2 ? 8 : 1);   // host bytes per device byte
        for (size_t off = 0; off < p.bytes; off += piece)
            ps.push_back({(const char*)p.d + off, (char*)p.h + off * scale, p.bytes - off < piece ? p.bytes - off : piece,
                          p.widen});
    }
    const size_t np = ps.size();
    auto issue = [&](size_t i) -> int {
        const int r = (int)(i % h.kRing);
        HIP_TRY(ctx, hipMemcpyAsync(h.pin_out[r], ps[i].d, ps[i].n, hipMemcpyDeviceToHost, h.s_d2h));
        HIP_TRY(ctx, hipEventRecord(h.ev_pin_out[r], h.s_d2h));
        return RSP_OK;
    };
    int rc;
    for (size_t i = 0; i < np && i < (size_t)h.kRing; ++i)
        if ((rc = issue(i))) return rc;
    for (size_t i = 0; i < np; ++i) {
        const int r = (int)(i % h.kRing);
        HIP_TRY(ctx, hipEventSynchronize(h.ev_pin_out[r]));
        if (h.pf) h.pf->wait(ps[i].h, ps[i].n * (ps[i].widen == 1 ? 2 : (ps[i].widen == 2 ? 8 : 1)));
        if (ps[i].widen == 1) pool.widen_f32((double*)ps[i].h, (const float*)h.pin_out[r], ps[i].n / 4);
        else if (ps[i].widen == 2) pool.widen_u8((double*)ps[i].h, (const uint8_t*)h.pin_out[r], ps[i].n);
        else pool.copy(ps[i].h, h.pin_out[r], ps[i].n);
        if (i + h.kRing < np && (rc = issue(i + h.kRing))) return rc;
    }
    return RSP_OK;
}

int rsp_set_host_pipeline(rsp_ctx* ctx, int64_t cpis_per_chunk, int32_t copy_threads) {
    if (!ctx) return fail(nullptr, RSP_ERR_ARG, "null ctx");
    if (cpis_per_chunk < 0 || copy_threads < 0 || copy_threads > 64)
        return fail(ctx, RSP_ERR_ARG, "rsp_set_host_pipeline: chunk %lld, threads %d", (long long)cpis_per_chunk,
                    (int)copy_threads);
    ctx->host_chunk = cpis_per_chunk;
    ctx->hp.threads = copy_threads;
    return RSP_OK;
}

static int host_chain(rsp_ctx* ctx, const void* echo, int32_t dtype, int32_t layout, int64_t P, int64_t R,
                      int64_t batch, const rsp_cfar_params* cfar, void* rdm_out, int32_t out_layout,
                      void* flag_out, void* flagV_out, bool f64);

// The host-buffer chain: float / byte outputs, or (f64) MATLAB's double outputs.
static int host_call(rsp_ctx* ctx, const void* echo, int32_t dtype, int32_t layout, int64_t P, int64_t R,
                     int64_t batch, const rsp_cfar_params* cfar, void* rdm_out, int32_t out_layout, void* flag_out,
                     void* flagV_out, bool f64) {
    if (!ctx) return fail(nullptr, RSP_ERR_ARG, "null ctx");
    int rc;
    try {
        rc = host_chain(ctx, echo, dtype, layout, P, R, batch, cfar, rdm_out, out_layout, flag_out, flagV_out, f64);
    } catch (const std::bad_alloc&) {
        rc = fail(ctx, RSP_ERR_NOMEM, "rsp_pc_mtd_cfar: host allocation failed");
    } catch (const std::exception& e) {
        rc = fail(ctx, RSP_ERR_NOMEM, "rsp_pc_mtd_cfar: host pipeline: %s", e.what());
    } catch (...) {
        rc = fail(ctx, RSP_ERR_NOMEM, "rsp_pc_mtd_cfar: host pipeline: unknown exception");
    }
    if (rc && ctx->hp.s_h2d) {
        // an error after chunks were issued: drain all three streams before returning, so the
        // next call's first H2D cannot overwrite an input slot a chain still reads, nor its
        // output staging race a D2H still in flight (the status stays the first error's)
        (void)hipStreamSynchronize(ctx->hp.s_h2d);
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipStreamSynchronize(ctx->hp.s_d2h);
    }
    return rc;
}

int rsp_pc_mtd_cfar(rsp_ctx* ctx, const void* echo, int32_t dtype, int32_t layout, int64_t P, int64_t R,
                    int64_t batch, const rsp_cfar_params* cfar, float* rdm_out, int32_t out_layout,
                    uint8_t* flag_out, uint8_t* flagV_out) {
    return host_call(ctx, echo, dtype, layout, P, R, batch, cfar, rdm_out, out_layout, flag_out, flagV_out, false);
}

int rsp_pc_mtd_cfar_f64(rsp_ctx* ctx, const void* echo, int32_t dtype, int32_t layout, int64_t P, int64_t R,
                        int64_t batch, const rsp_cfar_params* cfar, double* rdm_out, int32_t out_layout,
                        double* flag_out, double* flagV_out) {
    return host_call(ctx, echo, dtype, layout, P, R, batch, cfar, rdm_out, out_layout, flag_out, flagV_out, true);
}

// Dev-only host-path trace (environment RSP_HOST_TRACE=1): per call, host time of the setup, the
// input staging (narrowing + DMA issue), the chain enqueue, the output staging (waits + widening)
// and the final syncs, plus device time of the H2D / chain / D2H streams (timing events), on
// stderr.  Used by tools/mex_bench.py --trace to find where a one-CPI MEX call spends its time.
struct HostTrace {
    bool on = false;
    std::chrono::steady_clock::time_point t[8];
    int n = 0;
    hipEvent_t e[6] = {};
    double acc[4] = {};   // one-chunk path: input conversion, output waits, output conversion (us)
    void mark() { if (on && n < 8) t[n++] = std::chrono::steady_clock::now(); }
    double now_us() const {
        return on ? std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count() : 0.0;
    }
    void ev(int i, hipStream_t st) { if (on) (void)hipEventRecord(e[i], st); }
};
static bool host_trace_on() {
    static const bool on = [] { const char* v = getenv("RSP_HOST_TRACE"); return v && *v == '1'; }();
    return on;
}

// One-chunk calls (MATLAB's granularity: fun_MTD_produce is one CPI per call) are latency-bound,
// not bandwidth-bound: a pinned DMA pays ~13 us of fixed cost per copy and ~11 us more to
// signal the host (tools/micro/host_latency_probe.hip, profiles/r05/mex/), and the host's
// narrowing / widening sat between DMAs on the critical path.  Here the kernels move the data
// across PCIe themselves:
//   * input: the copy threads narrow (or copy) the caller's echo into pinned staging in pieces
//     of ~1 MiB that never cross a plane; right behind each piece, a transpose (column-major) or
//     copy (row-major) kernel on the chain's stream reads it from pinned memory into the
//     chain's device input -- PCIe transfer, ingest transpose and host narrowing overlap;
//   * output: after the chain, transpose / copy kernels write the RDM and flag planes into
//     pinned staging in up to kParts parts, an event behind each; the copy threads widen (or
//     copy) part q into the caller's arrays while parts q+1.. cross the link.
// Staging is allocated coherent (fine-grained: not cached in the GPU's L2), so a kernel never
// reads a previous call's input from L2 and the host never reads output lines the L2 still holds.
// RSP_HOST_ZC=0 (dev A/B) restores the DMA pipeline for every call.
static constexpr size_t kZcPiece = 1u << 20;       // device bytes per input piece
static constexpr size_t kZcMaxIn = 64u << 20;      // one-chunk calls up to this much device input
static int zc_knob(const char* name, int dflt) {   // dev A/B knobs of the one-chunk path
    const char* v = getenv(name);
    return v && *v ? atoi(v) : dflt;
}
static int zc_mode() {
    static const int m = [] { const char* v = getenv("RSP_HOST_ZC"); return v && *v ? atoi(v) : 1; }();
    return m;
}
static int zc_ensure(rsp_ctx* ctx, void** p, size_t* n, size_t bytes) {
    if (*p && *n >= bytes) return RSP_OK;
    if (*p) {
        HIP_TRY(ctx, hipHostFree(*p));
        *p = nullptr;
        *n = 0;
    }
    HIP_TRY(ctx, hipHostMalloc(p, bytes, zc_mode() == 2 ? hipHostMallocDefault : hipHostMallocCoherent));
    *n = bytes;
    return RSP_OK;
}

// Output delivery of the one-chunk paths: planes [batch][V][Ro] of each output (device, `es`
// bytes per element: 4 float, 1 byte) are transposed (tr: the caller's column-major [Ro][V]) or
// copied into pinned staging by kernels on ctx->stream, in parts of whole range-bin rows with an
// event behind each; the copy threads deliver part q -- widened to double when f64 -- into the
// caller's array while the later parts cross the link.
struct ZcOut {
    const void* dev;
    int es;
    void* host;
    bool f64;
};
static int zc_deliver(rsp_ctx* ctx, const ZcOut* outs, int nout, int64_t batch, int64_t V, int64_t Ro, bool tr,
                      HostTrace& ht) {
    auto& h = ctx->hp;
    const size_t cells = (size_t)V * Ro, ocells = (size_t)batch * cells;
    size_t bytes = 0;
    for (int k = 0; k < nout; ++k) bytes += ocells * outs[k].es;
    int rc;
    if ((rc = zc_ensure(ctx, &h.zc_out, &h.zc_out_n, bytes))) return rc;
    hipStream_t st = ctx->stream;
    struct Part {
        int k;
        size_t off, n;
    };
    Part parts[rsp_ctx::HostPipe::kParts];
    int np = 0;
    // parts of >= ~1 MiB of device output (a part costs a kernel and an event: at c3, 2 parts of
    // the 2 MiB RDM beat 4 of 512 KiB; executeCFAR's ~170 KB segments go whole), within kParts
    static const size_t kPartBytes = (size_t)zc_knob("RSP_ZC_PART_KIB", 1024) << 10;
    const int budget = h.kParts / (nout * (int)batch);
    char* zk[3] = {};
    size_t zoff = 0;
    for (int k = 0; k < nout; ++k) {
        zk[k] = (char*)h.zc_out + zoff;
        zoff += ocells * outs[k].es;
    }
    for (int k = 0; k < nout; ++k) {
        const size_t es = (size_t)outs[k].es;
        const int elem = es == 4 ? rsp::RSP_SUB_F32 : rsp::RSP_SUB_U8;
        int per_plane = (int)((cells * es + kPartBytes / 2) / kPartBytes);
        per_plane = per_plane < 1 ? 1 : (per_plane > budget ? budget : per_plane);
        if (tr) {   // plane b: [V][Ro] -> [Ro][V]; a part = output rows [c0, c1) (range bins)
            int64_t cp = (Ro + per_plane - 1) / per_plane;
            cp = (cp + 31) / 32 * 32;
            for (int64_t b = 0; b < batch; ++b)
                for (int64_t c0 = 0; c0 < Ro; c0 += cp) {
                    const int64_t c1 = c0 + cp < Ro ? c0 + cp : Ro;
                    HIP_TRY(ctx, rsp::launch_transpose_sub(elem, (const char*)outs[k].dev + ((size_t)b * cells + c0) * es,
                                                           zk[k] + (size_t)(b * Ro + c0) * V * es, (int)V, (int)(c1 - c0),
                                                           (size_t)Ro, (size_t)V, st));
                    HIP_TRY(ctx, hipEventRecord(h.ev_part[np], st));
                    parts[np++] = {k, (size_t)(b * Ro + c0) * V, (size_t)(c1 - c0) * V};
                }
        } else {    // row-major: contiguous parts (whole 4-byte words: ocells % 4 == 0, checked)
            const int nparts = per_plane * (int)batch;
            size_t pe = (ocells + nparts - 1) / nparts;
            pe = (pe + 1023) / 1024 * 1024;
            for (size_t off = 0; off < ocells; off += pe) {
                const size_t n = ocells - off < pe ? ocells - off : pe;
                HIP_TRY(ctx, rsp::launch_copy_words((const char*)outs[k].dev + off * es, zk[k] + off * es, n * es / 4, st));
                HIP_TRY(ctx, hipEventRecord(h.ev_part[np], st));
                parts[np++] = {k, off, n};
            }
        }
    }
    ht.mark();   // 3: chain and output kernels enqueued
    rsp::CopyPool& pool = host_pool(ctx);
    for (int q = 0; q < np; ++q) {
        const Part& pt = parts[q];
        const ZcOut& o = outs[pt.k];
        const double t0 = ht.now_us();
        HIP_TRY(ctx, hipEventSynchronize(h.ev_part[q]));
        const double t1 = ht.now_us();
        const char* zp = zk[pt.k] + pt.off * o.es;
        if (h.pf) h.pf->wait((char*)o.host + pt.off * (o.f64 ? 8 : o.es), pt.n * (o.f64 ? 8 : o.es));
        if (o.es == 4) {
            if (o.f64) pool.widen_f32((double*)o.host + pt.off, (const float*)zp, pt.n);
            else pool.copy((float*)o.host + pt.off, zp, pt.n * 4);
        } else {
            if (o.f64) pool.widen_u8((double*)o.host + pt.off, (const uint8_t*)zp, pt.n);
            else pool.copy((uint8_t*)o.host + pt.off, zp, pt.n);
        }
        ht.acc[1] += t1 - t0;
        ht.acc[2] += ht.now_us() - t1;
    }
    return RSP_OK;
}

static int host_chain_small(rsp_ctx* ctx, const void* echo, int32_t dtype, int32_t layout, int64_t P, int64_t R,
                            int64_t batch, const rsp_cfar_params* cfar, void* rdm_out, int32_t out_layout,
                            void* flag_out, void* flagV_out, bool f64, HostTrace& ht, bool& taken) {
    auto& h = ctx->hp;
    taken = false;
    const int64_t Ro = ctx->p.R_out, V = ctx->V, beams = ctx->beams;
    const bool narrow = dtype == RSP_C128;
    const int32_t ddtype = narrow ? RSP_C64 : dtype;
    const size_t ein = dtype_size(dtype), edev = dtype_size(ddtype);
    const bool conv = layout != RSP_ROWMAJOR, tr = out_layout == RSP_COLMAJOR;
    const bool want_fv = cfar && flagV_out;
    const int64_t planes = batch * beams;
    const size_t elems = (size_t)planes * P * R, dbytes = elems * edev;
    const size_t cells = (size_t)V * Ro, ocells = (size_t)batch * cells;
    const int nkinds = (rdm_out ? 1 : 0) + (cfar ? 1 : 0) + (want_fv ? 1 : 0);
    if (dbytes > kZcMaxIn || (int64_t)nkinds * batch > h.kParts || (!tr && (ocells % 4) != 0) ||
        (!conv && (dbytes % 4) != 0))
        return RSP_OK;   // not taken: the DMA pipeline runs the call
    taken = true;
    int rc;
    if ((rc = zc_ensure(ctx, &h.zc_in, &h.zc_in_n, dbytes))) return rc;
    if ((rc = ensure(ctx, h.in[0], dbytes))) return rc;
    if (conv && (rc = ensure(ctx, h.canon[0], elems * sizeof(float2)))) return rc;
    if ((rc = ensure(ctx, h.rdm[0], ocells * sizeof(float)))) return rc;
    if (cfar && (rc = ensure(ctx, h.flag[0], ocells))) return rc;
    if (want_fv && (rc = ensure(ctx, h.flagV[0], ocells))) return rc;
    rsp::CopyPool& pool = host_pool(ctx);
    hipStream_t st = ctx->stream;
    char* zin = (char*)h.zc_in;
    const char* src = (const char*)echo;
    // ---- input pieces: source elements [s0, s0 + n)
    auto stage = [&](size_t s0, size_t n) {
        const double t0 = ht.now_us();
        if (narrow) pool.narrow_c128((float*)(zin + s0 * edev), (const double*)(src + s0 * ein), n);
        else pool.copy(zin + s0 * edev, src + s0 * ein, n * edev);
        std::atomic_thread_fence(std::memory_order_release);
        ht.acc[0] += ht.now_us() - t0;
    };
    static const size_t kPiece = (size_t)zc_knob("RSP_ZC_PIECE_KIB", (int)(kZcPiece >> 10)) << 10;
    if (conv) {   // plane k = [R][P] -> canon [P][R]; a piece = rows [r0, r1) of one plane
        int64_t rp = (int64_t)(kPiece / ((size_t)P * edev)) / 32 * 32;
        if (rp < 32) rp = 32;
        const int elem = ddtype == RSP_C32F16 ? rsp::RSP_SUB_C32F16 : rsp::RSP_SUB_C64;
        for (int64_t k = 0; k < planes; ++k)
            for (int64_t r0 = 0; r0 < R; r0 += rp) {
                const int64_t r1 = r0 + rp < R ? r0 + rp : R;
                const size_t s0 = (size_t)(k * R + r0) * P;
                stage(s0, (size_t)(r1 - r0) * P);
                HIP_TRY(ctx, rsp::launch_transpose_sub(elem, zin + s0 * edev,
                                                       (float2*)h.canon[0].p + (size_t)k * P * R + r0, (int)(r1 - r0),
                                                       (int)P, (size_t)P, (size_t)R, st));
            }
    } else {      // row-major: contiguous pieces, copied as they are
        const size_t pe = (kPiece / edev + 1023) / 1024 * 1024;
        for (size_t s0 = 0; s0 < elems; s0 += pe) {
            const size_t n = elems - s0 < pe ? elems - s0 : pe;
            stage(s0, n);
            HIP_TRY(ctx, rsp::launch_copy_words(zin + s0 * edev, (char*)h.in[0].p + s0 * edev, n * edev / 4, st));
        }
    }
    ht.mark();   // 2: input staged
    ht.ev(2, st);
    int rc2 = rsp_pc_mtd_cfar_dev(ctx, conv ? h.canon[0].p : h.in[0].p, conv ? RSP_C64 : ddtype, batch, cfar,
                                  (float*)h.rdm[0].p, cfar ? (uint8_t*)h.flag[0].p : nullptr,
                                  want_fv ? (uint8_t*)h.flagV[0].p : nullptr, st);
    if (rc2) return rc2;
    ht.ev(3, st);
    ht.ev(4, st);
    ZcOut outs[3];
    int no = 0;
    if (rdm_out) outs[no++] = {h.rdm[0].p, 4, rdm_out, f64};
    if (cfar) outs[no++] = {h.flag[0].p, 1, flag_out, f64};
    if (want_fv) outs[no++] = {h.flagV[0].p, 1, flagV_out, f64};
    if ((rc = zc_deliver(ctx, outs, no, batch, V, Ro, tr, ht))) return rc;
    ht.ev(5, st);
    ht.mark();   // 4: outputs delivered
    return RSP_OK;
}

// Prefault of the caller's output arrays (rsp_hostpool.h Prefaulter) from the start of a call
// whose outputs total >= kPrefaultMin bytes: new arrays of that size are fresh anonymous
// mappings (glibc serves allocations above its mmap threshold, at most 32 MiB, by mmap), and
// the copy threads would otherwise take one page fault + zeroing per 4 KiB as they deliver.
// The job ends (workers off the caller's memory) before the call returns, on every path.
// Dev A/B: RSP_PREFAULT=0 off; RSP_PREFAULT_THREADS (default 4); RSP_PREFAULT_HUGE=0 (no
// MADV_HUGEPAGE advice).  (Faulting on the calling thread's NUMA node was measured neutral on the
// GPU box -- every page landed on node 0 either way, profiles/r06/host/numa_ab/ -- and is not
// kept.)
static constexpr size_t kPrefaultMin = 8u << 20;
struct PrefaultJob {
    rsp_ctx* ctx = nullptr;
    ~PrefaultJob() {
        if (ctx && ctx->hp.pf) {
            ctx->hp.pf->end();
            ctx->hp.pf = nullptr;
        }
    }
};
static void host_prefault(rsp_ctx* ctx, PrefaultJob& job, const std::vector<std::pair<void*, size_t>>& ranges) {
    static const int mode = zc_knob("RSP_PREFAULT", 1);
    static const int nthr = zc_knob("RSP_PREFAULT_THREADS", 4);
    static const int huge = zc_knob("RSP_PREFAULT_HUGE", 1);
    size_t total = 0;
    for (const auto& r : ranges) total += r.first ? r.second : 0;
    if (mode == 0 || total < kPrefaultMin) return;
    auto& h = ctx->hp;
    if (!h.prefault) h.prefault.reset(new rsp::Prefaulter(nthr, huge != 0));
    std::vector<std::pair<void*, size_t>> rs;
    for (const auto& r : ranges)
        if (r.first && r.second) rs.push_back(r);
    h.prefault->begin(rs);
    h.pf = h.prefault.get();
    job.ctx = ctx;
}

static int host_chain(rsp_ctx* ctx, const void* echo, int32_t dtype, int32_t layout, int64_t P, int64_t R,
                      int64_t batch, const rsp_cfar_params* cfar, void* rdm_out, int32_t out_layout,
                      void* flag_out, void* flagV_out, bool f64) {
    HostTrace ht;
    ht.on = host_trace_on();
    if (ht.on)
        for (auto& e : ht.e) (void)hipEventCreate(&e);
    ht.mark();
    int rc = check_host_call(ctx, echo, dtype, layout, P, R, batch);
    if (rc) return rc;
    if (out_layout != RSP_ROWMAJOR && out_layout != RSP_COLMAJOR) return fail(ctx, RSP_ERR_ARG, "bad out_layout");
    if (cfar && !flag_out) return fail(ctx, RSP_ERR_ARG, "CFAR requested without flag_out");
    if (!cfar && !rdm_out) return fail(ctx, RSP_ERR_ARG, "no output requested");
    if (batch == 0) return RSP_OK;
    if ((rc = host_pipe_init(ctx))) return rc;
    auto& h = ctx->hp;
    const int64_t Ro = ctx->p.R_out, V = ctx->V, beams = ctx->beams;
    // MATLAB's complex double is narrowed to complex float by the host copy threads (the same
    // round-to-nearest cast the device conversion does): half the PCIe bytes
    const bool narrow = dtype == RSP_C128;
    const int32_t ddtype = narrow ? RSP_C64 : dtype;              // what lands on the device
    const size_t in_cpi = (size_t)beams * P * R * dtype_size(dtype);         // caller's bytes
    const size_t dev_cpi = (size_t)beams * P * R * dtype_size(ddtype);       // device bytes
    const size_t cells = (size_t)V * Ro;   // per CPI
    const bool conv = layout != RSP_ROWMAJOR;   // column-major: transposed on the device
    const bool tr = out_layout == RSP_COLMAJOR;
    const bool want_fv = cfar && flagV_out;
    int64_t K = ctx->host_chunk > 0 ? ctx->host_chunk : (int64_t)(kHostChunkBytes / dev_cpi);
    if (K < 1) K = 1;
    if (K > batch) K = batch;
    const int64_t nk = (batch + K - 1) / K;
    PrefaultJob pfjob;   // (ends the prefault job on every return below)
    {
        const size_t oc = (size_t)batch * cells, rb = f64 ? 8 : 4, fb = f64 ? 8 : 1;
        host_prefault(ctx, pfjob, {{rdm_out, rdm_out ? oc * rb : 0}, {flag_out, cfar ? oc * fb : 0},
                                   {flagV_out, want_fv ? oc * fb : 0}});
    }
    if (nk == 1 && zc_mode() != 0) {
        ht.mark();   // 1: set up
        bool taken = false;
        rc = host_chain_small(ctx, echo, dtype, layout, P, R, batch, cfar, rdm_out, out_layout, flag_out, flagV_out,
                              f64, ht, taken);
        if (taken) {
            if (rc == RSP_OK && ht.on) {
                ht.mark();   // 5
                (void)hipStreamSynchronize(ctx->stream);
                float g[2] = {};
                (void)hipEventElapsedTime(&g[0], ht.e[2], ht.e[3]);
                (void)hipEventElapsedTime(&g[1], ht.e[4], ht.e[5]);
                auto us = [&](int a, int b) { return std::chrono::duration<double, std::micro>(ht.t[b] - ht.t[a]).count(); };
                fprintf(stderr, "rsp_host_trace batch %lld chunks 1 zc host_us setup %.1f stage_in %.1f enqueue %.1f "
                        "stage_out %.1f sync %.1f total %.1f dev_us h2d 0 chain %.1f d2h %.1f zc_us narrow %.1f "
                        "wait %.1f widen %.1f\n", (long long)batch,
                        us(0, 1), us(1, 2), us(2, 3), us(3, 4), us(4, 5), us(0, 5), g[0] * 1e3, g[1] * 1e3, ht.acc[0],
                        ht.acc[1], ht.acc[2]);
            }
            if (ht.on)
                for (auto& e : ht.e) (void)hipEventDestroy(e);
            return rc;
        }
        ht.n = 1;   // (the DMA pipeline's marks follow)
    }
    for (int i = 0; i < h.kSlots && i < nk; ++i) {
        if ((rc = ensure(ctx, h.in[i], (size_t)K * dev_cpi))) return rc;
        if (conv && (rc = ensure(ctx, h.canon[i], (size_t)K * beams * P * R * sizeof(float2)))) return rc;
        if ((rc = ensure(ctx, h.rdm[i], (size_t)K * cells * sizeof(float)))) return rc;
        if (cfar && (rc = ensure(ctx, h.flag[i], (size_t)K * cells))) return rc;
        if (want_fv && (rc = ensure(ctx, h.flagV[i], (size_t)K * cells))) return rc;
        if (tr) {
            if (rdm_out && (rc = ensure(ctx, h.tr[i][0], (size_t)K * cells * sizeof(float)))) return rc;
            if (cfar && (rc = ensure(ctx, h.tr[i][1], (size_t)K * cells))) return rc;
            if (want_fv && (rc = ensure(ctx, h.tr[i][2], (size_t)K * cells))) return rc;
        }
    }
    // chunk k: the chain on slot k % 2 after its H2D, then transposes; its outputs' D2H waits for it
    auto chunk_n = [&](int64_t k) { return k == nk - 1 ? batch - k * K : K; };
    auto compute = [&](int64_t k) -> int {
        const int sl = (int)(k % h.kSlots);
        const int64_t n = chunk_n(k);
        HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, h.ev_in[sl], 0));
        if (k >= h.kSlots) HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, h.ev_out[sl], 0));   // slot's D2H done
        const void* d_echo = h.in[sl].p;
        int32_t d_dtype = ddtype;
        if (conv) {
            HIP_TRY(ctx, rsp::launch_ingest(h.in[sl].p, ddtype, layout, (float2*)h.canon[sl].p, n * beams, (int)P,
                                            (int)R, ctx->stream));
            d_echo = h.canon[sl].p;
            d_dtype = RSP_C64;
        }
        int rc2 = rsp_pc_mtd_cfar_dev(ctx, d_echo, d_dtype, n, cfar, (float*)h.rdm[sl].p,
                                      cfar ? (uint8_t*)h.flag[sl].p : nullptr,
                                      want_fv ? (uint8_t*)h.flagV[sl].p : nullptr, ctx->stream);
        if (rc2) return rc2;
        if (tr) {
            if (rdm_out)
                HIP_TRY(ctx, rsp::launch_transpose_f32((const float*)h.rdm[sl].p, (float*)h.tr[sl][0].p, n, (int)V,
                                                       (int)Ro, ctx->stream));
            if (cfar)
                HIP_TRY(ctx, rsp::launch_transpose_u8((const uint8_t*)h.flag[sl].p, (uint8_t*)h.tr[sl][1].p, n, (int)V,
                                                      (int)Ro, ctx->stream));
            if (want_fv)
                HIP_TRY(ctx, rsp::launch_transpose_u8((const uint8_t*)h.flagV[sl].p, (uint8_t*)h.tr[sl][2].p, n,
                                                      (int)V, (int)Ro, ctx->stream));
        }
        HIP_TRY(ctx, hipEventRecord(h.ev_comp[sl], ctx->stream));
        return RSP_OK;
    };
    auto output = [&](int64_t k) -> int {
        const int sl = (int)(k % h.kSlots);
        const size_t n = (size_t)chunk_n(k), o = (size_t)k * K * cells;
        HIP_TRY(ctx, hipStreamWaitEvent(h.s_d2h, h.ev_comp[sl], 0));
        std::vector<D2HPart> parts;
        const size_t rb = f64 ? 8 : 4, fb = f64 ? 8 : 1;   // host bytes per RDM / flag element
        if (rdm_out)
            parts.push_back({tr ? h.tr[sl][0].p : h.rdm[sl].p, (char*)rdm_out + o * rb, n * cells * sizeof(float), f64 ? 1 : 0});
        if (cfar) parts.push_back({tr ? h.tr[sl][1].p : h.flag[sl].p, (char*)flag_out + o * fb, n * cells, f64 ? 2 : 0});
        if (want_fv)
            parts.push_back({tr ? h.tr[sl][2].p : h.flagV[sl].p, (char*)flagV_out + o * fb, n * cells, f64 ? 2 : 0});
        int rc2 = d2h_pieces(ctx, parts);
        if (rc2) return rc2;
        HIP_TRY(ctx, hipEventRecord(h.ev_out[sl], h.s_d2h));
        return RSP_OK;
    };
    ht.mark();   // 1: set up
    for (int64_t k = 0; k < nk; ++k) {
        const int sl = (int)(k % h.kSlots);
        // the slot's previous chain (chunk k-2) has read its input
        if (k >= h.kSlots) HIP_TRY(ctx, hipStreamWaitEvent(h.s_h2d, h.ev_comp[sl], 0));
        if (k == 0) ht.ev(0, h.s_h2d);
        if ((rc = h2d_pieces(ctx, h.in[sl].p, (const char*)echo + (size_t)k * K * in_cpi, (size_t)chunk_n(k) * dev_cpi,
                             narrow ? 1 : 0)))
            return rc;
        if (k == nk - 1) ht.ev(1, h.s_h2d);
        HIP_TRY(ctx, hipEventRecord(h.ev_in[sl], h.s_h2d));
        if (k == 0) ht.mark();   // 2: first chunk staged
        if (k == 0) {
            HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, h.ev_in[sl], 0));
            ht.ev(2, ctx->stream);
        }
        if ((rc = compute(k))) return rc;
        if (k == nk - 1) ht.ev(3, ctx->stream);
        if (k == 0) ht.mark();   // 3: first chain enqueued
        if (k >= 1 && (rc = output(k - 1))) return rc;
    }
    if (ht.on) {
        HIP_TRY(ctx, hipStreamWaitEvent(h.s_d2h, h.ev_comp[(nk - 1) % h.kSlots], 0));
        ht.ev(4, h.s_d2h);
    }
    if ((rc = output(nk - 1))) return rc;
    ht.ev(5, h.s_d2h);
    ht.mark();   // 4: outputs staged
    HIP_TRY(ctx, hipStreamSynchronize(h.s_d2h));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    ht.mark();   // 5: done
    if (ht.on) {
        float g[3] = {};
        (void)hipEventElapsedTime(&g[0], ht.e[0], ht.e[1]);
        (void)hipEventElapsedTime(&g[1], ht.e[2], ht.e[3]);
        (void)hipEventElapsedTime(&g[2], ht.e[4], ht.e[5]);
        auto us = [&](int a, int b) { return std::chrono::duration<double, std::micro>(ht.t[b] - ht.t[a]).count(); };
        fprintf(stderr, "rsp_host_trace batch %lld chunks %lld host_us setup %.1f stage_in %.1f enqueue %.1f stage_out %.1f "
                "sync %.1f total %.1f dev_us h2d %.1f chain %.1f d2h %.1f\n", (long long)batch, (long long)nk, us(0, 1),
                us(1, 2), us(2, 3), us(3, 4), us(4, 5), us(0, 5), g[0] * 1e3, g[1] * 1e3, g[2] * 1e3);
        for (auto& e : ht.e) (void)hipEventDestroy(e);
    }
    return RSP_OK;
}

int rsp_pc_mtd(rsp_ctx* ctx, const void* echo, int32_t dtype, int32_t layout, int64_t P, int64_t R,
               int64_t batch, float* rdm_out, int32_t rdm_layout) {
    if (!rdm_out) return fail(ctx, RSP_ERR_ARG, "rsp_pc_mtd: null rdm_out");
    return rsp_pc_mtd_cfar(ctx, echo, dtype, layout, P, R, batch, nullptr, rdm_out, rdm_layout, nullptr, nullptr);
}

int rsp_cfar(rsp_ctx* ctx, const float* rdm, int32_t rdm_layout, int64_t V, int64_t R, int64_t batch,
             const rsp_cfar_params* cfar, uint8_t* flag_out, uint8_t* flagV_out) {
    if (!ctx) return fail(nullptr, RSP_ERR_ARG, "null ctx");
    if (!rdm || !cfar || !flag_out || V < 1 || R < 1 || batch < 0) return fail(ctx, RSP_ERR_ARG, "rsp_cfar: bad argument");
    if (rdm_layout != RSP_ROWMAJOR && rdm_layout != RSP_COLMAJOR) return fail(ctx, RSP_ERR_ARG, "bad rdm_layout");
    if (batch == 0) return RSP_OK;
    if (!set_device(ctx)) return fail(ctx, RSP_ERR_HIP, "hipSetDevice failed");
    const size_t cells = (size_t)batch * V * R;
    int rc;
    if ((rc = ensure(ctx, ctx->st_in, cells * sizeof(float)))) return rc;
    if ((rc = ensure(ctx, ctx->st_rdm, cells * sizeof(float)))) return rc;
    if ((rc = ensure(ctx, ctx->st_flag, cells))) return rc;
    if ((rc = ensure(ctx, ctx->st_flagV, cells))) return rc;
    HIP_TRY(ctx, hipMemcpyAsync(ctx->st_in.p, rdm, cells * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
    const float* d_rdm = (const float*)ctx->st_in.p;
    if (rdm_layout == RSP_COLMAJOR) {  // MATLAB V x R = [b][R][V] -> [b][V][R]
        HIP_TRY(ctx, rsp::launch_transpose_f32(d_rdm, (float*)ctx->st_rdm.p, batch, (int)R, (int)V, ctx->stream));
        d_rdm = (const float*)ctx->st_rdm.p;
    }
    rc = rsp_cfar_dev(ctx, d_rdm, V, R, batch, cfar, (uint8_t*)ctx->st_flag.p, (uint8_t*)ctx->st_flagV.p, ctx->stream);
    if (rc) return rc;
    if ((rc = fetch(ctx, (const uint8_t*)ctx->st_flag.p, flag_out, batch, V, R, rdm_layout))) return rc;
    if (flagV_out && (rc = fetch(ctx, (const uint8_t*)ctx->st_flagV.p, flagV_out, batch, V, R, rdm_layout)))
        return rc;
    return RSP_OK;
}

// executeCFAR with MATLAB's types (rsp.h): the double RDM narrowed to float by the copy pool on
// its way into the pinned input ring, the 0/1 flags widened to double as their pieces land.
static int cfar_f64_body(rsp_ctx* ctx, const double* rdm, int32_t rdm_layout, int64_t V, int64_t R, int64_t batch,
                         const rsp_cfar_params* cfar, double* flag_out, double* flagV_out) {
    int rc;
    if ((rc = host_pipe_init(ctx))) return rc;
    const size_t cells = (size_t)batch * V * R;
    if ((rc = ensure(ctx, ctx->st_in, cells * sizeof(float)))) return rc;
    if ((rc = ensure(ctx, ctx->st_rdm, cells * sizeof(float)))) return rc;
    if ((rc = ensure(ctx, ctx->st_flag, cells))) return rc;
    if ((rc = ensure(ctx, ctx->st_flagV, cells))) return rc;
    auto& h = ctx->hp;
    const bool col = rdm_layout == RSP_COLMAJOR;
    if (zc_mode() != 0 && cells * sizeof(float) <= kZcMaxIn && (flagV_out ? 2 : 1) * batch <= h.kParts &&
        (col || cells % 4 == 0)) {
        // one chunk (executeCFAR's segments): the narrowed pieces are read from pinned staging by
        // the transpose / copy kernels, the flags written back into it part by part (host_chain_small)
        if ((rc = zc_ensure(ctx, &h.zc_in, &h.zc_in_n, cells * sizeof(float)))) return rc;
        rsp::CopyPool& pool = host_pool(ctx);
        char* zin = (char*)h.zc_in;
        hipStream_t st = ctx->stream;
        if (col) {   // plane k = [R][V] -> [V][R]; a piece = rows [r0, r1) of one plane
            int64_t rp = (int64_t)(kZcPiece / ((size_t)V * sizeof(float))) / 32 * 32;
            if (rp < 32) rp = 32;
            for (int64_t k = 0; k < batch; ++k)
                for (int64_t r0 = 0; r0 < R; r0 += rp) {
                    const int64_t r1 = r0 + rp < R ? r0 + rp : R;
                    const size_t s0 = (size_t)(k * R + r0) * V;
                    pool.narrow_f64((float*)zin + s0, rdm + s0, (size_t)(r1 - r0) * V);
                    std::atomic_thread_fence(std::memory_order_release);
                    HIP_TRY(ctx, rsp::launch_transpose_sub(rsp::RSP_SUB_F32, (float*)zin + s0,
                                                           (float*)ctx->st_rdm.p + (size_t)k * V * R + r0, (int)(r1 - r0),
                                                           (int)V, (size_t)V, (size_t)R, st));
                }
        } else {
            const size_t pe = kZcPiece / sizeof(float);
            for (size_t s0 = 0; s0 < cells; s0 += pe) {
                const size_t n = cells - s0 < pe ? cells - s0 : pe;
                pool.narrow_f64((float*)zin + s0, rdm + s0, n);
                std::atomic_thread_fence(std::memory_order_release);
                HIP_TRY(ctx, rsp::launch_copy_words((float*)zin + s0, (float*)ctx->st_in.p + s0, n, st));
            }
        }
        rc = rsp_cfar_dev(ctx, (const float*)(col ? ctx->st_rdm.p : ctx->st_in.p), V, R, batch, cfar,
                          (uint8_t*)ctx->st_flag.p, (uint8_t*)ctx->st_flagV.p, st);
        if (rc) return rc;
        ZcOut outs[2] = {{ctx->st_flag.p, 1, flag_out, true}, {ctx->st_flagV.p, 1, flagV_out, true}};
        HostTrace none;
        return zc_deliver(ctx, outs, flagV_out ? 2 : 1, batch, V, R, col, none);
    }
    if ((rc = h2d_pieces(ctx, ctx->st_in.p, rdm, cells * sizeof(float), 2))) return rc;
    HIP_TRY(ctx, hipEventRecord(h.ev_in[0], h.s_h2d));
    HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, h.ev_in[0], 0));
    const float* d_rdm = (const float*)ctx->st_in.p;
    if (col) {  // MATLAB V x R = [b][R][V] -> [b][V][R]
        HIP_TRY(ctx, rsp::launch_transpose_f32(d_rdm, (float*)ctx->st_rdm.p, batch, (int)R, (int)V, ctx->stream));
        d_rdm = (const float*)ctx->st_rdm.p;
    }
    rc = rsp_cfar_dev(ctx, d_rdm, V, R, batch, cfar, (uint8_t*)ctx->st_flag.p, (uint8_t*)ctx->st_flagV.p, ctx->stream);
    if (rc) return rc;
    const uint8_t* f = (const uint8_t*)ctx->st_flag.p;
    const uint8_t* fv = (const uint8_t*)ctx->st_flagV.p;
    if (col) {   // back to MATLAB's [b][R][V]
        if ((rc = ensure(ctx, ctx->st_t, cells))) return rc;
        if ((rc = ensure(ctx, ctx->st_canon, cells))) return rc;
        HIP_TRY(ctx, rsp::launch_transpose_u8(f, (uint8_t*)ctx->st_t.p, batch, (int)V, (int)R, ctx->stream));
        f = (const uint8_t*)ctx->st_t.p;
        if (flagV_out) {
            HIP_TRY(ctx, rsp::launch_transpose_u8(fv, (uint8_t*)ctx->st_canon.p, batch, (int)V, (int)R, ctx->stream));
            fv = (const uint8_t*)ctx->st_canon.p;
        }
    }
    HIP_TRY(ctx, hipEventRecord(h.ev_comp[0], ctx->stream));
    HIP_TRY(ctx, hipStreamWaitEvent(h.s_d2h, h.ev_comp[0], 0));
    std::vector<D2HPart> parts;
    parts.push_back({f, flag_out, cells, 2});
    if (flagV_out) parts.push_back({fv, flagV_out, cells, 2});
    if ((rc = d2h_pieces(ctx, parts))) return rc;
    HIP_TRY(ctx, hipStreamSynchronize(h.s_d2h));
    return RSP_OK;
}

int rsp_cfar_f64(rsp_ctx* ctx, const double* rdm, int32_t rdm_layout, int64_t V, int64_t R, int64_t batch,
                 const rsp_cfar_params* cfar, double* flag_out, double* flagV_out) {
    if (!ctx) return fail(nullptr, RSP_ERR_ARG, "null ctx");
    if (!rdm || !cfar || !flag_out || V < 1 || R < 1 || batch < 0) return fail(ctx, RSP_ERR_ARG, "rsp_cfar_f64: bad argument");
    if (rdm_layout != RSP_ROWMAJOR && rdm_layout != RSP_COLMAJOR) return fail(ctx, RSP_ERR_ARG, "bad rdm_layout");
    if (batch == 0) return RSP_OK;
    if (!set_device(ctx)) return fail(ctx, RSP_ERR_HIP, "hipSetDevice failed");
    int rc;
    try {
        rc = cfar_f64_body(ctx, rdm, rdm_layout, V, R, batch, cfar, flag_out, flagV_out);
    } catch (const std::exception& e) {
        rc = fail(ctx, RSP_ERR_NOMEM, "rsp_cfar_f64: host pipeline: %s", e.what());
    } catch (...) {
        rc = fail(ctx, RSP_ERR_NOMEM, "rsp_cfar_f64: host pipeline: unknown exception");
    }
    if (rc && ctx->hp.s_h2d) {
        (void)hipStreamSynchronize(ctx->hp.s_h2d);
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipStreamSynchronize(ctx->hp.s_d2h);
    }
    return rc;
}

