/*
 * executeCFAR_mex.c -- MEX drop-in for
 *   [flag, flagV] = executeCFAR(rdm, refR, saveR, TR, mR, refV, saveV, TV, mV, M0, rFlag)
 * (MatlabProcess_xuzerui/CFAR_WangCai/executeCFAR.m:1-2).  fun_CFARflag is a local
 * function of main_cfar.m (:142) and cannot be shadowed, so the interposition point is
 * executeCFAR, which fun_CFARflag calls once per column segment (:147-154).
 *
 * Build:  mex -R2018a -I<repo>/include executeCFAR_mex.c \
 *             -L<repo>/radar-signal-process_amd/lib -lrsp -output executeCFAR
 * rdm: V x R real double (column-major, converted to fp32 for the GPU).  Outputs are
 * V x R double 0/1 like the reference.  A CFAR window that does not fit raises
 * rsp:cfar_window, as MATLAB's index error would.
 */
#include <string.h>

#include <stdlib.h>

#include "mex.h"
#include "rsp.h"

static rsp_ctx* g_ctx = NULL;

/* GPU of the shim's context: RSP_MEX_DEVICE (a HIP device index, default 0), read when the
 * context is created (first call, or a call whose parameters change); setenv('RSP_MEX_DEVICE',
 * '3') in MATLAB before that call places it on device 3.  One MATLAB process drives one GPU. */
static int mex_device(void) {
    const char* d = getenv("RSP_MEX_DEVICE");
    return d && *d ? atoi(d) : 0;
}

static void cleanup(void) {
    if (g_ctx) rsp_destroy(g_ctx);
    g_ctx = NULL;
}

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs != 11)
        mexErrMsgIdAndTxt("rsp:usage", "[flag, flagV] = executeCFAR(rdm, refR, saveR, TR, mR, refV, saveV, TV, mV, M0, rFlag)");
    const mxArray* M = prhs[0];
    if (!mxIsDouble(M) || mxIsComplex(M)) mexErrMsgIdAndTxt("rsp:rdm", "rdm must be real double");
    const int64_t V = (int64_t)mxGetM(M), R = (int64_t)mxGetN(M);
    rsp_cfar_params cf;
    memset(&cf, 0, sizeof(cf));
    cf.refR = (int32_t)mxGetScalar(prhs[1]);
    cf.saveR = (int32_t)mxGetScalar(prhs[2]);
    cf.TR = mxGetScalar(prhs[3]);
    cf.methodR = (int32_t)mxGetScalar(prhs[4]);
    cf.refV = (int32_t)mxGetScalar(prhs[5]);
    cf.saveV = (int32_t)mxGetScalar(prhs[6]);
    cf.TV = mxGetScalar(prhs[7]);
    cf.methodV = (int32_t)mxGetScalar(prhs[8]);
    cf.M0 = (int32_t)mxGetScalar(prhs[9]);
    cf.rFlag = mxGetScalar(prhs[10]) != 0.0;
    cf.zero_v_div = 0;
    cf.nseg = 0;
    if (!g_ctx) {
        if (rsp_create(&g_ctx, mex_device(), NULL) != RSP_OK) {
            g_ctx = NULL;
            mexErrMsgIdAndTxt("rsp:create", "%s", rsp_last_error(NULL));
        }
        mexAtExit(cleanup);
    }
    /* double in, double 0/1 out: the narrowing and widening run on the library's copy threads,
     * piece by piece beside the DMA (rsp_cfar_f64).  Every flag element is written, so the
     * outputs skip MATLAB's zero fill (mxCreateUninitNumericMatrix, R2015a+) */
    plhs[0] = mxCreateUninitNumericMatrix((size_t)V, (size_t)R, mxDOUBLE_CLASS, mxREAL);
    mxArray* fv = nlhs > 1 ? mxCreateUninitNumericMatrix((size_t)V, (size_t)R, mxDOUBLE_CLASS, mxREAL) : NULL;
    if (!plhs[0] || (nlhs > 1 && !fv)) {
        if (plhs[0]) mxDestroyArray(plhs[0]);
        plhs[0] = NULL;
        if (fv) mxDestroyArray(fv);
        mexErrMsgIdAndTxt("rsp:nomem", "cannot allocate the %lld x %lld flag planes", (long long)V, (long long)R);
    }
    int rc = rsp_cfar_f64(g_ctx, mxGetDoubles(M), RSP_COLMAJOR, V, R, 1, &cf, mxGetDoubles(plhs[0]),
                          fv ? mxGetDoubles(fv) : NULL);
    if (rc != RSP_OK) {
        char msg[512];
        strncpy(msg, rsp_last_error(g_ctx), sizeof(msg) - 1);
        msg[sizeof(msg) - 1] = 0;
        mxDestroyArray(plhs[0]);
        plhs[0] = NULL;
        if (fv) mxDestroyArray(fv);
        mexErrMsgIdAndTxt(rc == RSP_ERR_CFAR_WINDOW ? "rsp:cfar_window" : "rsp:run", "%s", msg);
    }
    if (fv) plhs[1] = fv;
}
