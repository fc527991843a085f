/*
 * fun_MTD_produce_mex.c -- MEX drop-in for MTD_Signal = fun_MTD_produce(echoData, params)
 * (MTD/fun_MTD_produce.m:12; called at MTD/main_produce_dataset_win_xzr_v2.m:136).
 *
 * Build (MATLAB R2018a+ interleaved complex API), output named so it shadows the .m file:
 *   mex -R2018a -I<repo>/include fun_MTD_produce_mex.c \
 *       -L<repo>/radar-signal-process_amd/lib -lrsp -output fun_MTD_produce
 * echoData: P x R complex double (MATLAB column-major; passed to the library as-is,
 * RSP_C128 + RSP_COLMAJOR, converted on the GPU).  params: the v2 struct (prtNum, fs, B,
 * tao(3), point_prt(4); other fields ignored, debug plotting is not reproduced).
 * Returns the P x R real double RDM.  One context is cached per parameter set and freed
 * at mexAtExit; library errors become mexErrMsgIdAndTxt("rsp:...") after cleanup.
 */
#include <string.h>

#include "mex.h"
#include "rsp.h"

static rsp_ctx* g_ctx = NULL;
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

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    (void)nlhs;
    if (nrhs != 2) mexErrMsgIdAndTxt("rsp:usage", "MTD_Signal = fun_MTD_produce(echoData, params)");
    const mxArray* E = prhs[0];
    if (!mxIsDouble(E) || !mxIsComplex(E)) mexErrMsgIdAndTxt("rsp:echo", "echoData must be complex double");
    if (!mxIsStruct(prhs[1])) mexErrMsgIdAndTxt("rsp:params", "params must be a struct");
    const int64_t P = (int64_t)mxGetM(E), R = (int64_t)mxGetN(E);
    const double* pp = mxGetDoubles(need_field(prhs[1], "point_prt", 4));
    const double* tao = mxGetDoubles(need_field(prhs[1], "tao", 3));
    const double fs = mxGetScalar(need_field(prhs[1], "fs", 1));
    const double B = mxGetScalar(need_field(prhs[1], "B", 1));
    double key[12] = {(double)P, (double)R, pp[0], pp[1], pp[2], pp[3], fs, B, tao[0], tao[1], tao[2], 0.0};
    if (!g_ctx || memcmp(key, g_key, sizeof(key)) != 0) {
        cleanup();
        int64_t point_prt[4] = {R, (int64_t)pp[1], (int64_t)pp[2], (int64_t)pp[3]};
        if (rsp_create_v2(&g_ctx, 0, P, R, point_prt, fs, B, tao) != RSP_OK) {
            g_ctx = NULL;
            mexErrMsgIdAndTxt("rsp:create", "%s", rsp_last_error(NULL));
        }
        memcpy(g_key, key, sizeof(key));
        mexAtExit(cleanup);
    }
    float* rdm = (float*)mxMalloc((size_t)(P * R) * sizeof(float));
    int rc = rsp_pc_mtd(g_ctx, mxGetComplexDoubles(E), RSP_C128, RSP_COLMAJOR, P, R, 1, rdm, RSP_COLMAJOR);
    if (rc != RSP_OK) {
        char msg[512];
        strncpy(msg, rsp_last_error(g_ctx), sizeof(msg) - 1);
        msg[sizeof(msg) - 1] = 0;
        mxFree(rdm);
        mexErrMsgIdAndTxt("rsp:run", "%s", msg);
    }
    plhs[0] = mxCreateDoubleMatrix((mwSize)P, (mwSize)R, mxREAL);
    double* out = mxGetDoubles(plhs[0]);
    for (int64_t i = 0; i < P * R; ++i) out[i] = rdm[i];
    mxFree(rdm);
}
