/* A minimal fake of the MATLAB MEX runtime (the functions tests/mex_stub/mex.h declares),
 * linked with one MEX shim from radar-signal-process_amd/mex into a shared library, so the
 * shim's mexFunction runs from Python (tests/test_mex_runtime.py) on the GPU box exactly as
 * MATLAB would call it: column-major double arrays (complex interleaved, R2018a API), structs
 * with named fields, mexErrMsgIdAndTxt unwinding to the caller, mexAtExit cleanups.
 * Test infrastructure only -- MATLAB is not installed here or on the GPU box. */
#include <setjmp.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mex.h"

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]);

struct mxArray_tag {
    int is_struct, is_complex;
    size_t m, n;
    double* re;                 /* real doubles, or interleaved (re, im) pairs when complex */
    int nfields;
    char** names;
    mxArray** values;
};

static jmp_buf g_jmp;
static int g_in_call = 0;
static char g_errid[128], g_errmsg[1024];
static void (*g_atexit[16])(void);
static int g_natexit = 0;

/* ---- MEX API (as the shims use it) ---- */
int mxIsDouble(const mxArray* a) { return a && !a->is_struct; }
int mxIsComplex(const mxArray* a) { return a && a->is_complex; }
int mxIsStruct(const mxArray* a) { return a && a->is_struct; }
size_t mxGetM(const mxArray* a) { return a->m; }
size_t mxGetN(const mxArray* a) { return a->n; }
size_t mxGetNumberOfElements(const mxArray* a) { return a->m * a->n; }
mxArray* mxGetField(const mxArray* s, size_t i, const char* name) {
    if (!s || !s->is_struct || i != 0) return NULL;
    for (int k = 0; k < s->nfields; ++k)
        if (strcmp(s->names[k], name) == 0) return s->values[k];
    return NULL;
}
double mxGetScalar(const mxArray* a) { return (a && a->re && a->m * a->n > 0) ? a->re[0] : 0.0; }
double* mxGetDoubles(const mxArray* a) { return (a && !a->is_complex) ? a->re : NULL; }
mxComplexDouble* mxGetComplexDoubles(const mxArray* a) { return (a && a->is_complex) ? (mxComplexDouble*)a->re : NULL; }
mxArray* mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity c) {
    mxArray* a = (mxArray*)calloc(1, sizeof(mxArray));
    a->m = m;
    a->n = n;
    a->is_complex = c == mxCOMPLEX;
    a->re = (double*)calloc(m * n * (a->is_complex ? 2 : 1) + 1, sizeof(double));
    return a;
}
/* MATLAB's uninitialised allocation (R2015a+): the same array without the zero fill -- in
 * this fake, malloc instead of calloc (only mxDOUBLE_CLASS, the one class the shims create) */
mxArray* mxCreateUninitNumericMatrix(size_t m, size_t n, mxClassID cls, mxComplexity c) {
    if (cls != mxDOUBLE_CLASS) return NULL;
    mxArray* a = (mxArray*)calloc(1, sizeof(mxArray));
    a->m = m;
    a->n = n;
    a->is_complex = c == mxCOMPLEX;
    a->re = (double*)malloc((m * n * (a->is_complex ? 2 : 1) + 1) * sizeof(double));
    return a;
}
void* mxMalloc(size_t n) { return malloc(n); }
void mxFree(void* p) { free(p); }
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...) {
    snprintf(g_errid, sizeof(g_errid), "%s", id);
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_errmsg, sizeof(g_errmsg), fmt, ap);
    va_end(ap);
    if (g_in_call) longjmp(g_jmp, 1);
    abort();   /* outside rt_call: nothing to unwind to */
}
int mexAtExit(void (*fn)(void)) {
    for (int i = 0; i < g_natexit; ++i)
        if (g_atexit[i] == fn) return 0;
    if (g_natexit < 16) g_atexit[g_natexit++] = fn;
    return 0;
}

/* ---- harness side (ctypes) ---- */
mxArray* rt_double(size_t m, size_t n, const double* data, int is_complex) {
    mxArray* a = mxCreateDoubleMatrix(m, n, is_complex ? mxCOMPLEX : mxREAL);
    if (data) memcpy(a->re, data, m * n * (is_complex ? 2 : 1) * sizeof(double));
    return a;
}
mxArray* rt_struct(int nfields, const char** names, mxArray** values) {
    mxArray* s = (mxArray*)calloc(1, sizeof(mxArray));
    s->is_struct = 1;
    s->m = s->n = 1;
    s->nfields = nfields;
    s->names = (char**)calloc((size_t)nfields, sizeof(char*));
    s->values = (mxArray**)calloc((size_t)nfields, sizeof(mxArray*));
    for (int k = 0; k < nfields; ++k) {
        s->names[k] = (char*)malloc(strlen(names[k]) + 1);
        strcpy(s->names[k], names[k]);
        s->values[k] = values[k];   /* the struct takes ownership */
    }
    return s;
}
void rt_free(mxArray* a) {
    if (!a) return;
    for (int k = 0; k < a->nfields; ++k) {
        free(a->names[k]);
        rt_free(a->values[k]);
    }
    free(a->names);
    free(a->values);
    free(a->re);
    free(a);
}
void mxDestroyArray(mxArray* a) { rt_free(a); }
size_t rt_m(const mxArray* a) { return a->m; }
size_t rt_n(const mxArray* a) { return a->n; }
int rt_is_complex(const mxArray* a) { return a->is_complex; }
const double* rt_data(const mxArray* a) { return a->re; }
const char* rt_errid(void) { return g_errid; }
const char* rt_errmsg(void) { return g_errmsg; }

/* Call the shim's mexFunction; 0 on success, 1 if it raised (rt_errid / rt_errmsg).  Output
 * arrays a raising call created before the raise are not reported (MATLAB discards them). */
int rt_call(int nlhs, mxArray** plhs, int nrhs, mxArray** prhs) {
    g_errid[0] = g_errmsg[0] = 0;
    for (int i = 0; i < nlhs; ++i) plhs[i] = NULL;
    g_in_call = 1;
    if (setjmp(g_jmp) != 0) {
        g_in_call = 0;
        return 1;
    }
    mexFunction(nlhs, plhs, nrhs, (const mxArray**)prhs);
    g_in_call = 0;
    return 0;
}

/* "clear mex": run the registered mexAtExit cleanups */
void rt_clear(void) {
    for (int i = g_natexit - 1; i >= 0; --i) g_atexit[i]();
    g_natexit = 0;
}
