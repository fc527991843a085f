/* A plain C program over the C ABI (include/rsp.h), as a C caller of the reference's hot path
 * binds it -- no Python, no torch.  Run by tests/test_gpu_capi_consumer.py on the GPU box.
 *
 * One v2 context at 128 x 4096 (fun_MTD_produce's params, MTD/main_produce_dataset_win_xzr_v2.m:
 * 31-45), a CPI of complex noise plus one moving point target (the 28 us pulse3 chirp echoed at
 * range column TGT of segment 3, a Doppler phase ramp of FD cycles over the P pulses), in
 * MATLAB's layout (complex double, column-major), and:
 *   - rsp_pc_mtd_cfar (float / byte outputs) in both input layouts and both output layouts:
 *     identical outputs;
 *   - rsp_pc_mtd_cfar_f64 and rsp_pc_mtd (fun_MTD_produce): the same values;
 *   - rsp_cfar_f64 on the double RDM (executeCFAR): the chain's flags;
 *   - the target: the RDM maximum lies on Doppler row FD + P/2 (the fftshift) and range column
 *     TGT (the matched filter's peak at the echo's first sample), and the CFAR flags it;
 *   - rsp_set_range_concat (fun_lss_range_concate): the RDM of two concatenated column ranges is
 *     the full RDM's columns gathered, bit for bit; a part past the width is RSP_ERR_ARG; 0 parts
 *     restore the full width;
 *   - the error contract: a wrong shape is RSP_ERR_SHAPE with a message, a null context
 *     RSP_ERR_ARG.
 * Prints "ok <peak row> <peak column> <detections>" and exits 0, or prints the failed check
 * and exits 1. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rsp.h"

#define P 128
#define R 4096
#define FD 20
#define TGT 1800

static int fails = 0;
#define CHECK(c, ...)                    \
    do {                                 \
        if (!(c)) {                      \
            printf("FAIL: " __VA_ARGS__); \
            printf("\n");                \
            ++fails;                     \
        }                                \
    } while (0)

static uint64_t rng = 0x9e3779b97f4a7c15ull;
static double uni(void) {   /* (0, 1] */
    rng = rng * 6364136223846793005ull + 1442695040888963407ull;
    return ((rng >> 11) + 1) * (1.0 / 9007199254740992.0);
}
static double gauss(void) { return sqrt(-2.0 * log(uni())) * cos(2.0 * M_PI * uni()); }

int main(void) {
    const int64_t pp[4] = {R, 228, 723, R - 951};
    const double fs = 25e6, B = 20e6, tao[3] = {0.16e-6, 8e-6, 28e-6};
    rsp_ctx* ctx = NULL;
    if (rsp_create_v2(&ctx, 0, P, R, pp, fs, B, tao) != RSP_OK) {
        printf("FAIL: rsp_create_v2: %s\n", rsp_last_error(NULL));
        return 1;
    }
    const size_t n = (size_t)P * R;
    double* col = malloc(2 * n * sizeof(double));   /* MATLAB P x R: element (p, r) at r*P + p */
    double* row = malloc(2 * n * sizeof(double));   /* [P][R] */
    for (size_t i = 0; i < 2 * n; ++i) col[i] = gauss() * sqrt(0.5);
    const int L = (int)lround(tao[2] * fs);          /* 700 chirp samples */
    for (int p = 0; p < P; ++p)
        for (int k = 0; k < L && TGT + k < R; ++k) {
            const double t = -tao[2] / 2 + k / fs;
            const double ph = M_PI * (B / tao[2]) * t * t + 2.0 * M_PI * FD * p / P;
            const size_t e = (size_t)(TGT + k) * P + p;
            col[2 * e] += 4.0 * cos(ph);
            col[2 * e + 1] += 4.0 * sin(ph);
        }
    for (int p = 0; p < P; ++p)
        for (int r = 0; r < R; ++r) {
            row[2 * ((size_t)p * R + r)] = col[2 * ((size_t)r * P + p)];
            row[2 * ((size_t)p * R + r) + 1] = col[2 * ((size_t)r * P + p) + 1];
        }
    rsp_cfar_params cf;
    memset(&cf, 0, sizeof(cf));
    cf.refR = 5; cf.saveR = 7; cf.TR = 4.0; cf.methodR = 0;   /* main_cfar.m:40-58 */
    cf.refV = 5; cf.saveV = 7; cf.TV = 4.0; cf.methodV = 0;
    cf.M0 = 3; cf.rFlag = 1; cf.zero_v_div = 20;
    float *rdm = malloc(n * 4), *rdm_c = malloc(n * 4), *rdm2 = malloc(n * 4);
    uint8_t *fl = malloc(n), *fv = malloc(n), *fl_c = malloc(n), *fv_c = malloc(n);
    int rc = rsp_pc_mtd_cfar(ctx, row, RSP_C128, RSP_ROWMAJOR, P, R, 1, &cf, rdm, RSP_ROWMAJOR, fl, fv);
    CHECK(rc == RSP_OK, "rsp_pc_mtd_cfar row-major: %d %s", rc, rsp_last_error(ctx));
    rc = rsp_pc_mtd_cfar(ctx, col, RSP_C128, RSP_COLMAJOR, P, R, 1, &cf, rdm_c, RSP_COLMAJOR, fl_c, fv_c);
    CHECK(rc == RSP_OK, "rsp_pc_mtd_cfar column-major: %d %s", rc, rsp_last_error(ctx));
    int same = 1;
    for (int v = 0; v < P && same; ++v)
        for (int r = 0; r < R; ++r) {
            const size_t a = (size_t)v * R + r, b = (size_t)r * P + v;
            if (rdm[a] != rdm_c[b] || fl[a] != fl_c[b] || fv[a] != fv_c[b]) { same = 0; break; }
        }
    CHECK(same, "row-major and column-major calls differ");
    rc = rsp_pc_mtd(ctx, row, RSP_C128, RSP_ROWMAJOR, P, R, 1, rdm2, RSP_ROWMAJOR);
    CHECK(rc == RSP_OK && memcmp(rdm2, rdm, n * 4) == 0, "rsp_pc_mtd RDM differs from the chain's (%d)", rc);
    double *r64 = malloc(n * 8), *f64 = malloc(n * 8), *v64 = malloc(n * 8);
    rc = rsp_pc_mtd_cfar_f64(ctx, col, RSP_C128, RSP_COLMAJOR, P, R, 1, &cf, r64, RSP_COLMAJOR, f64, v64);
    CHECK(rc == RSP_OK, "rsp_pc_mtd_cfar_f64: %d %s", rc, rsp_last_error(ctx));
    same = 1;
    for (size_t i = 0; i < n; ++i)
        if (r64[i] != (double)rdm_c[i] || f64[i] != (double)fl_c[i] || v64[i] != (double)fv_c[i]) { same = 0; break; }
    CHECK(same, "the double outputs differ from the float / byte outputs");
    /* executeCFAR on the double RDM (CFAR-only context): the chain's flags */
    rsp_ctx* cctx = NULL;
    rc = rsp_create(&cctx, 0, NULL);
    CHECK(rc == RSP_OK, "rsp_create (CFAR only): %s", rsp_last_error(NULL));
    if (rc == RSP_OK) {
        double *cf64 = malloc(n * 8), *cv64 = malloc(n * 8);
        rc = rsp_cfar_f64(cctx, r64, RSP_COLMAJOR, P, R, 1, &cf, cf64, cv64);
        CHECK(rc == RSP_OK, "rsp_cfar_f64: %d %s", rc, rsp_last_error(cctx));
        CHECK(rc != RSP_OK || (memcmp(cf64, f64, n * 8) == 0 && memcmp(cv64, v64, n * 8) == 0),
              "rsp_cfar_f64 on the chain's RDM differs from the chain's flags");
        free(cf64);
        free(cv64);
        rsp_destroy(cctx);
    }
    /* the target */
    size_t best = 0;
    for (size_t i = 1; i < n; ++i)
        if (rdm[i] > rdm[best]) best = i;
    const int bv = (int)(best / R), br = (int)(best % R);
    long det = 0;
    for (size_t i = 0; i < n; ++i) det += fl[i];
    CHECK(bv == FD + P / 2, "RDM peak on Doppler row %d, expected %d", bv, FD + P / 2);
    /* the matched filter ifft(fft(x) .* conj(fft(h))) peaks at the echo's first sample */
    CHECK(br >= TGT - 1 && br <= TGT + 1, "RDM peak at range column %d, the echo starts at %d", br, TGT);
    int flagged = 0;
    for (int dr = -1; dr <= 1; ++dr)
        if (br + dr >= 0 && br + dr < R && fl[(size_t)bv * R + br + dr]) flagged = 1;
    CHECK(flagged, "the CFAR does not flag the target (row %d, column %d)", bv, br);
    /* range concatenation (fun_lss_range_concate): the MTD transforms each range column on its
     * own, so the concatenated RDM is the full RDM's columns gathered, bit for bit -- the second
     * part holds the target */
    {
        const int64_t cs[2] = {3000, 1000}, cl[2] = {600, 1200}, W = 1800;
        float* rdm_k = malloc((size_t)P * W * 4);
        rc = rsp_set_range_concat(ctx, 2, cs, cl);
        CHECK(rc == RSP_OK, "rsp_set_range_concat: %d %s", rc, rsp_last_error(ctx));
        rc = rsp_pc_mtd(ctx, row, RSP_C128, RSP_ROWMAJOR, P, R, 1, rdm_k, RSP_ROWMAJOR);
        CHECK(rc == RSP_OK, "rsp_pc_mtd after concat: %d %s", rc, rsp_last_error(ctx));
        same = rc == RSP_OK;
        for (int v = 0; v < P && same; ++v)
            for (int64_t j = 0; j < W; ++j) {
                const int64_t src = j < cl[0] ? cs[0] + j : cs[1] + j - cl[0];
                if (rdm_k[(size_t)v * W + j] != rdm[(size_t)v * R + src]) { same = 0; break; }
            }
        CHECK(same, "the concatenated RDM is not the full RDM's gathered columns");
        const int64_t bs[1] = {R - 10}, bl[1] = {20};
        rc = rsp_set_range_concat(ctx, 1, bs, bl);
        CHECK(rc == RSP_ERR_ARG && strlen(rsp_last_error(ctx)) > 0, "a part past the PC width: status %d", rc);
        rc = rsp_set_range_concat(ctx, 0, NULL, NULL);
        CHECK(rc == RSP_OK, "rsp_set_range_concat(0 parts): %d", rc);
        rc = rsp_pc_mtd(ctx, row, RSP_C128, RSP_ROWMAJOR, P, R, 1, rdm2, RSP_ROWMAJOR);
        CHECK(rc == RSP_OK && memcmp(rdm2, rdm, n * 4) == 0, "the full width is not restored (%d)", rc);
        free(rdm_k);
    }
    /* error contract */
    rc = rsp_pc_mtd_cfar(ctx, row, RSP_C128, RSP_ROWMAJOR, P + 1, R, 1, &cf, rdm, RSP_ROWMAJOR, fl, fv);
    CHECK(rc == RSP_ERR_SHAPE && strlen(rsp_last_error(ctx)) > 0, "wrong P: status %d", rc);
    rc = rsp_pc_mtd_cfar(NULL, row, RSP_C128, RSP_ROWMAJOR, P, R, 1, &cf, rdm, RSP_ROWMAJOR, fl, fv);
    CHECK(rc == RSP_ERR_ARG, "null context: status %d", rc);
    rsp_destroy(ctx);
    free(col); free(row); free(rdm); free(rdm_c); free(rdm2); free(fl); free(fv); free(fl_c); free(fv_c);
    free(r64); free(f64); free(v64);
    if (fails) return 1;
    printf("ok %d %d %ld\n", bv, br, det);
    return 0;
}
