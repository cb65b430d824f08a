/*
 * mex.h — TEST-ONLY minimal stand-in for MATLAB's MEX/mx API (R2018a
 * interleaved-complex interface), just the calls integration/matlab/ntm_mpc_mex.c
 * makes.  MATLAB is not in this image; this lets the gateway's argument
 * parsing, array layout and error paths be compiled and driven from the tests
 * (tests/test_mex_gateway.py).  It is not a MATLAB replacement and never ships.
 */
#ifndef NTM_TEST_MEX_H
#define NTM_TEST_MEX_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum { mxUNKNOWN_CLASS = 0, mxSTRUCT_CLASS, mxCHAR_CLASS, mxDOUBLE_CLASS, mxINT32_CLASS } mxClassID;
typedef enum { mxREAL = 0, mxCOMPLEX = 1 } mxComplexity;
typedef struct mxArray_tag mxArray;

void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...) __attribute__((noreturn));
int mexAtExit(void (*fn)(void));

mxArray* mxCreateDoubleMatrix(size_t m, size_t n, mxComplexity c);
mxArray* mxCreateNumericMatrix(size_t m, size_t n, mxClassID cls, mxComplexity c);
mxArray* mxDuplicateArray(const mxArray* a);
void mxDestroyArray(mxArray* a);
mxArray* mxGetField(const mxArray* s, size_t i, const char* name);
int mxIsDouble(const mxArray* a);
int mxIsInt32(const mxArray* a);
int mxIsChar(const mxArray* a);
int mxIsStruct(const mxArray* a);
int mxIsComplex(const mxArray* a);
size_t mxGetM(const mxArray* a);
size_t mxGetN(const mxArray* a);
size_t mxGetNumberOfElements(const mxArray* a);
double* mxGetDoubles(const mxArray* a);
int32_t* mxGetInt32s(const mxArray* a);
double mxGetScalar(const mxArray* a);
int mxGetString(const mxArray* a, char* buf, size_t n);

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]);

#ifdef __cplusplus
}
#endif
#endif
