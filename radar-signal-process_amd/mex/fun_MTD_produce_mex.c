/*
 * fun_MTD_produce_mex.c -- MEX drop-in for both forms of fun_MTD_produce:
 *   MTD_Signal = fun_MTD_produce(echoData, params)   v2 (MTD/fun_MTD_produce.m:12; called at
 *                                                    MTD/main_produce_dataset_win_xzr_v2.m:136)
 *   MTD_Signal = fun_MTD_produce(echo)               legacy (MatlabProcess_xuzerui/fun_MTD_produce.m:3;
 *                                                    called at main_produce_dataset_win_xzr.m:37-38
 *                                                    and MTD/main_produce_dataset_win_xzr_v1.m:105)
 *
 * Build (MATLAB R2018a+ interleaved complex API), output named so it shadows the .m file:
 *   mex -R2018a -I<repo>/include -DRSP_DATA_DIR='"<repo>/radar-signal-process_amd/rsp/data"' \
 *       fun_MTD_produce_mex.c -L<repo>/radar-signal-process_amd/lib -lrsp -output fun_MTD_produce
 * echoData: P x R complex double (MATLAB column-major; passed to the library as-is,
 * RSP_C128 + RSP_COLMAJOR, converted on the GPU).  params: the v2 struct (prtNum, fs, B,
 * tao(3), point_prt(4); other fields ignored, debug plotting is not reproduced).
 * The legacy form takes its two measured pulses from legacy_pulse2.npy / legacy_pulse3.npy in
 * $RSP_DATA_DIR (or the compile-time RSP_DATA_DIR): complex128 vectors extracted from the .m
 * file by tools/extract_reference_data.py.
 * Returns the P x R real double RDM.  One context is cached per parameter set and freed
 * at mexAtExit; library errors become mexErrMsgIdAndTxt("rsp:...") after cleanup.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mex.h"
#include "rsp.h"

#ifndef RSP_DATA_DIR
#define RSP_DATA_DIR "radar-signal-process_amd/rsp/data"
#endif

static rsp_ctx* g_ctx = NULL;

/* GPU of the shim's context: RSP_MEX_DEVICE (a HIP device index, default 0), read when the
 * context is created (first call, or a call whose parameters change); setenv('RSP_MEX_DEVICE',
 * '3') in MATLAB before that call places it on device 3.  One MATLAB process drives one GPU. */
static int mex_device(void) {
    const char* d = getenv("RSP_MEX_DEVICE");
    return d && *d ? atoi(d) : 0;
}
static double g_key[12];

static void cleanup(void) {
    if (g_ctx) rsp_destroy(g_ctx);
    g_ctx = NULL;
}

static const mxArray* need_field(const mxArray* s, const char* name, size_t n) {
    const mxArray* f = mxGetField(s, 0, name);
    if (!f || !mxIsDouble(f) || mxGetNumberOfElements(f) < n)
        mexErrMsgIdAndTxt("rsp:params", "params.%s missing or too short", name);
    return f;
}

/* A 1-D little-endian complex128 .npy vector (format 1.0/2.0, C order) into re / im arrays
 * (malloc'd).  Returns 0, or -1 with a message in err. */
static int read_npy_c128(const char* path, double** re, double** im, int64_t* n, char* err, size_t errn) {
    FILE* f = fopen(path, "rb");
    if (!f) { snprintf(err, errn, "cannot open %s", path); return -1; }
    unsigned char pre[12];
    int rc = -1;
    char* hdr = NULL;
    double* buf = NULL;
    if (fread(pre, 1, 10, f) != 10 || memcmp(pre, "\x93NUMPY", 6) != 0) {
        snprintf(err, errn, "%s: not an .npy file", path);
        goto done;
    }
    size_t hlen = (size_t)pre[8] | ((size_t)pre[9] << 8);
    if (pre[6] >= 2) {
        if (fread(pre + 10, 1, 2, f) != 2) goto done;
        hlen |= ((size_t)pre[10] << 16) | ((size_t)pre[11] << 24);
    }
    hdr = (char*)malloc(hlen + 1);
    if (!hdr || fread(hdr, 1, hlen, f) != hlen) { snprintf(err, errn, "%s: short header", path); goto done; }
    hdr[hlen] = 0;
    const char* sh = strstr(hdr, "'shape': (");
    if (!strstr(hdr, "'<c16'") || strstr(hdr, "'fortran_order': True") || !sh) {
        snprintf(err, errn, "%s: expected a C-order complex128 vector", path);
        goto done;
    }
    long long len = atoll(sh + 10);
    if (len < 1 || strchr(sh + 10, ',') != strchr(sh + 10, ')') - 1) {   /* "(N,)" only */
        snprintf(err, errn, "%s: expected a 1-D vector", path);
        goto done;
    }
    buf = (double*)malloc((size_t)len * 2 * sizeof(double));
    if (!buf || fread(buf, 2 * sizeof(double), (size_t)len, f) != (size_t)len) {
        snprintf(err, errn, "%s: short data", path);
        goto done;
    }
    *re = (double*)malloc((size_t)len * sizeof(double));
    *im = (double*)malloc((size_t)len * sizeof(double));
    if (!*re || !*im) { free(*re); free(*im); *re = *im = NULL; goto done; }
    for (long long i = 0; i < len; ++i) {
        (*re)[i] = buf[2 * i];
        (*im)[i] = buf[2 * i + 1];
    }
    *n = (int64_t)len;
    rc = 0;
done:
    free(buf);
    free(hdr);
    fclose(f);
    return rc;
}

static int create_legacy(int64_t P, int64_t R, char* err, size_t errn) {
    const char* dir = getenv("RSP_DATA_DIR");
    if (!dir || !*dir) dir = RSP_DATA_DIR;
    char path[1024];
    double *re2 = NULL, *im2 = NULL, *re3 = NULL, *im3 = NULL;
    int64_t n2 = 0, n3 = 0;
    int rc = -1;
    snprintf(path, sizeof(path), "%s/legacy_pulse2.npy", dir);
    if (read_npy_c128(path, &re2, &im2, &n2, err, errn) == 0) {
        snprintf(path, sizeof(path), "%s/legacy_pulse3.npy", dir);
        if (read_npy_c128(path, &re3, &im3, &n3, err, errn) == 0) {
            if (rsp_create_legacy(&g_ctx, mex_device(), P, R, re2, im2, n2, re3, im3, n3) == RSP_OK) rc = 0;
            else { g_ctx = NULL; snprintf(err, errn, "%s", rsp_last_error(NULL)); }
        }
    }
    free(re2); free(im2); free(re3); free(im3);
    return rc;
}

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    (void)nlhs;
    if (nrhs != 1 && nrhs != 2)
        mexErrMsgIdAndTxt("rsp:usage", "MTD_Signal = fun_MTD_produce(echoData, params) or fun_MTD_produce(echo)");
    const mxArray* E = prhs[0];
    if (!mxIsDouble(E) || !mxIsComplex(E)) mexErrMsgIdAndTxt("rsp:echo", "echoData must be complex double");
    if (nrhs == 2 && !mxIsStruct(prhs[1])) mexErrMsgIdAndTxt("rsp:params", "params must be a struct");
    const int64_t P = (int64_t)mxGetM(E), R = (int64_t)mxGetN(E);
    double key[12] = {(double)P, (double)R, 0, 0, 0, 0, 0, 0, 0, 0, 0, (double)nrhs};
    const double *pp = NULL, *tao = NULL;
    double fs = 0, B = 0;
    if (nrhs == 2) {
        pp = mxGetDoubles(need_field(prhs[1], "point_prt", 4));
        tao = mxGetDoubles(need_field(prhs[1], "tao", 3));
        fs = mxGetScalar(need_field(prhs[1], "fs", 1));
        B = mxGetScalar(need_field(prhs[1], "B", 1));
        const double k2[10] = {pp[0], pp[1], pp[2], pp[3], fs, B, tao[0], tao[1], tao[2]};
        memcpy(key + 2, k2, 9 * sizeof(double));
    }
    if (!g_ctx || memcmp(key, g_key, sizeof(key)) != 0) {
        cleanup();
        char err[512] = "";
        if (nrhs == 2) {
            int64_t point_prt[4] = {R, (int64_t)pp[1], (int64_t)pp[2], (int64_t)pp[3]};
            if (rsp_create_v2(&g_ctx, mex_device(), P, R, point_prt, fs, B, tao) != RSP_OK) {
                g_ctx = NULL;
                mexErrMsgIdAndTxt("rsp:create", "%s", rsp_last_error(NULL));
            }
        } else if (create_legacy(P, R, err, sizeof(err)) != 0) {
            mexErrMsgIdAndTxt("rsp:create", "%s", err);
        }
        memcpy(g_key, key, sizeof(key));
        mexAtExit(cleanup);
    }
    /* the RDM lands in MATLAB's double matrix directly: the library widens each device->host
     * piece on its copy threads as the piece arrives (rsp_pc_mtd_cfar_f64, cfar = NULL).  The
     * library writes every element, so the matrix is created without MATLAB's zero fill
     * (mxCreateUninitNumericMatrix, R2015a+): a zeroed P x R double is 4 MiB of memset per call
     * at 128 x 4096 */
    plhs[0] = mxCreateUninitNumericMatrix((size_t)P, (size_t)R, mxDOUBLE_CLASS, mxREAL);
    if (!plhs[0]) mexErrMsgIdAndTxt("rsp:nomem", "cannot allocate the %lld x %lld RDM", (long long)P, (long long)R);
    int rc = rsp_pc_mtd_cfar_f64(g_ctx, mxGetComplexDoubles(E), RSP_C128, RSP_COLMAJOR, P, R, 1, NULL,
                                 mxGetDoubles(plhs[0]), RSP_COLMAJOR, NULL, NULL);
    if (rc != RSP_OK) {
        char msg[512];
        strncpy(msg, rsp_last_error(g_ctx), sizeof(msg) - 1);
        msg[sizeof(msg) - 1] = 0;
        mxDestroyArray(plhs[0]);
        plhs[0] = NULL;
        mexErrMsgIdAndTxt("rsp:run", "%s", msg);
    }
}
