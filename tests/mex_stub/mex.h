/* Minimal stand-in declarations of the MATLAB MEX C API (R2018a interleaved complex),
 * used ONLY to compile-check the MEX shims in radar-signal-process_amd/mex here -- MATLAB is not
 * installed in this container or on the GPU box.  Not a MATLAB header. */
#ifndef RSP_TEST_MEX_STUB_H
#define RSP_TEST_MEX_STUB_H
#include <stddef.h>
#include <stdint.h>
typedef struct mxArray_tag mxArray;
typedef size_t mwSize;
typedef struct { double real, imag; } mxComplexDouble;
typedef enum { mxREAL = 0, mxCOMPLEX = 1 } mxComplexity;
typedef enum { mxUNKNOWN_CLASS = 0, mxDOUBLE_CLASS = 6 } mxClassID;
int mxIsDouble(const mxArray*);
int mxIsComplex(const mxArray*);
int mxIsStruct(const mxArray*);
size_t mxGetM(const mxArray*);
size_t mxGetN(const mxArray*);
size_t mxGetNumberOfElements(const mxArray*);
mxArray* mxGetField(const mxArray*, size_t, const char*);
double mxGetScalar(const mxArray*);
double* mxGetDoubles(const mxArray*);
mxComplexDouble* mxGetComplexDoubles(const mxArray*);
mxArray* mxCreateDoubleMatrix(mwSize, mwSize, mxComplexity);
mxArray* mxCreateUninitNumericMatrix(size_t, size_t, mxClassID, mxComplexity);
void* mxMalloc(size_t);
void mxFree(void*);
void mxDestroyArray(mxArray*);
void mexErrMsgIdAndTxt(const char*, const char*, ...);
int mexAtExit(void (*)(void));
#endif
