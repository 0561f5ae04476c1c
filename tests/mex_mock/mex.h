/* TEST INFRASTRUCTURE: a minimal stand-in for MATLAB's mex.h / matrix.h, enough to compile
 * and exercise colaborativempc-_amd/mex/cmpc_quadprog_mex.c and cmpc_lpv_mex.c without MATLAB (there is none
 * in this image).  Doubles only (full or sparse CSC), column-major, struct arrays of one element,
 * char arrays (command strings). */
#ifndef CMPC_MEX_MOCK_H
#define CMPC_MEX_MOCK_H
#include <stddef.h>

typedef size_t mwSize;
typedef size_t mwIndex;
typedef enum { mxDOUBLE_CLASS = 6, mxSTRUCT_CLASS = 2, mxCHAR_CLASS = 4 } mxClassID;
typedef enum { mxREAL = 0, mxCOMPLEX = 1 } mxComplexity;
typedef struct mxArray_tag mxArray;

mwSize mxGetNumberOfDimensions(const mxArray* a);
const mwSize* mxGetDimensions(const mxArray* a);
size_t mxGetNumberOfElements(const mxArray* a);
size_t mxGetM(const mxArray* a);
size_t mxGetN(const mxArray* a);
double* mxGetPr(const mxArray* a);
int mxIsDouble(const mxArray* a);
int mxIsComplex(const mxArray* a);
int mxIsSparse(const mxArray* a);
mwIndex* mxGetIr(const mxArray* a);
mwIndex* mxGetJc(const mxArray* a);
int mxGetNumberOfFields(const mxArray* a);
int mxIsEmpty(const mxArray* a);
int mxIsStruct(const mxArray* a);
int mxIsChar(const mxArray* a);
int mxGetString(const mxArray* a, char* buf, size_t buflen);
double mxGetScalar(const mxArray* a);
mxArray* mxGetField(const mxArray* a, size_t i, const char* name);
void mxSetField(mxArray* a, size_t i, const char* name, mxArray* v);
mxArray* mxCreateDoubleMatrix(size_t m, size_t n, mxComplexity c);
mxArray* mxCreateNumericArray(mwSize nd, const mwSize* dims, mxClassID cls, mxComplexity c);
mxArray* mxCreateStructMatrix(size_t m, size_t n, int nfields, const char** names);
mxArray* mxCreateString(const char* s);
void* mxCalloc(size_t n, size_t size);
void mxFree(void* p);
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...);
int mexAtExit(void (*fn)(void));
int mexPrintf(const char* fmt, ...);
#endif
