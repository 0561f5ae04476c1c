/* TEST INFRASTRUCTURE: implementation of the mock mex.h plus a ctypes-friendly harness
 * (mock_*) that builds argument arrays, calls mexFunction and reads results back.
 * mexErrMsgIdAndTxt longjmps back to mock_call, which reports the error id/message. */
#include <setjmp.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mex.h"

#define MAXF 32
struct mxArray_tag {
    mxClassID cls;
    mwSize nd;
    mwSize dims[4];
    double* pr;
    int nfields;
    char names[MAXF][32];
    mxArray* fields[MAXF];
    char* str;
    int sparse;          /* CSC: pr holds the nonzeros, ir their rows, jc the column starts */
    mwIndex *ir, *jc;
};

static jmp_buf g_jmp;
static char g_err_id[128], g_err_msg[512];
static void (*g_atexit)(void) = NULL;

mwSize mxGetNumberOfDimensions(const mxArray* a) { return a->nd; }
const mwSize* mxGetDimensions(const mxArray* a) { return a->dims; }
size_t mxGetNumberOfElements(const mxArray* a) {
    size_t k = 1;
    for (mwSize i = 0; i < a->nd; ++i) k *= a->dims[i];
    return k;
}
size_t mxGetM(const mxArray* a) { return a->dims[0]; }
size_t mxGetN(const mxArray* a) {
    size_t k = 1;
    for (mwSize i = 1; i < a->nd; ++i) k *= a->dims[i];
    return k;
}
double* mxGetPr(const mxArray* a) { return a->pr; }
int mxIsDouble(const mxArray* a) { return a->cls == mxDOUBLE_CLASS; }
int mxIsComplex(const mxArray* a) { (void)a; return 0; }
int mxIsSparse(const mxArray* a) { return a->sparse; }
mwIndex* mxGetIr(const mxArray* a) { return a->ir; }
mwIndex* mxGetJc(const mxArray* a) { return a->jc; }
int mxGetNumberOfFields(const mxArray* a) { return a->nfields; }
int mxIsEmpty(const mxArray* a) { return mxGetNumberOfElements(a) == 0; }
int mxIsStruct(const mxArray* a) { return a->cls == mxSTRUCT_CLASS; }
int mxIsChar(const mxArray* a) { return a->cls == mxCHAR_CLASS; }
/* MATLAB: 0 on success, 1 if not a char array or the buffer is too small */
int mxGetString(const mxArray* a, char* buf, size_t buflen) {
    if (a->cls != mxCHAR_CLASS || !a->str || strlen(a->str) + 1 > buflen) return 1;
    strcpy(buf, a->str);
    return 0;
}
double mxGetScalar(const mxArray* a) { return a->pr && mxGetNumberOfElements(a) ? a->pr[0] : 0.0; }
mxArray* mxGetField(const mxArray* a, size_t i, const char* name) {
    (void)i;
    for (int k = 0; k < a->nfields; ++k)
        if (!strcmp(a->names[k], name)) return a->fields[k];
    return NULL;
}
void mxSetField(mxArray* a, size_t i, const char* name, mxArray* v) {
    (void)i;
    for (int k = 0; k < a->nfields; ++k)
        if (!strcmp(a->names[k], name)) a->fields[k] = v;
}
mxArray* mxCreateNumericArray(mwSize nd, const mwSize* dims, mxClassID cls, mxComplexity c) {
    (void)c;
    mxArray* a = (mxArray*)calloc(1, sizeof(mxArray));
    a->cls = cls;
    a->nd = nd;
    for (mwSize i = 0; i < nd; ++i) a->dims[i] = dims[i];
    size_t k = mxGetNumberOfElements(a);
    a->pr = (double*)calloc(k ? k : 1, sizeof(double));
    return a;
}
mxArray* mxCreateDoubleMatrix(size_t m, size_t n, mxComplexity c) {
    mwSize d[2] = {m, n};
    return mxCreateNumericArray(2, d, mxDOUBLE_CLASS, c);
}
mxArray* mxCreateStructMatrix(size_t m, size_t n, int nfields, const char** names) {
    mxArray* a = (mxArray*)calloc(1, sizeof(mxArray));
    a->cls = mxSTRUCT_CLASS;
    a->nd = 2;
    a->dims[0] = m;
    a->dims[1] = n;
    a->nfields = nfields;
    for (int k = 0; k < nfields && k < MAXF; ++k) strncpy(a->names[k], names[k], 31);
    return a;
}
mxArray* mxCreateString(const char* s) {
    mxArray* a = mxCreateDoubleMatrix(1, strlen(s), mxREAL);
    a->cls = mxCHAR_CLASS;
    a->str = strdup(s);
    return a;
}
void* mxCalloc(size_t n, size_t size) { return calloc(n, size); }
void mxFree(void* p) { free(p); }
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err_msg, sizeof(g_err_msg), fmt, ap);
    va_end(ap);
    strncpy(g_err_id, id, sizeof(g_err_id) - 1);
    longjmp(g_jmp, 1);
}
int mexAtExit(void (*fn)(void)) {
    g_atexit = fn;
    return 0;
}
int mexPrintf(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    int r = vprintf(fmt, ap);
    va_end(ap);
    return r;
}

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]);

/* ---- harness ---- */
mxArray* mock_array(int nd, const long* dims, const double* data) {
    mwSize d[4] = {0, 0, 1, 1};
    for (int i = 0; i < nd && i < 4; ++i) d[i] = (mwSize)dims[i];
    mxArray* a = mxCreateNumericArray(nd, d, mxDOUBLE_CLASS, mxREAL);
    size_t k = mxGetNumberOfElements(a);
    if (data && k) memcpy(a->pr, data, k * sizeof(double));
    return a;
}
/* m x n sparse double in CSC form (nnz values, their row indices, n+1 column starts) */
mxArray* mock_sparse(long m, long n, long nnz, const double* pr, const long* ir, const long* jc) {
    mxArray* a = (mxArray*)calloc(1, sizeof(mxArray));
    a->cls = mxDOUBLE_CLASS;
    a->nd = 2;
    a->dims[0] = (mwSize)m;
    a->dims[1] = (mwSize)n;
    a->sparse = 1;
    a->pr = (double*)calloc(nnz ? nnz : 1, sizeof(double));
    a->ir = (mwIndex*)calloc(nnz ? nnz : 1, sizeof(mwIndex));
    a->jc = (mwIndex*)calloc(n + 1, sizeof(mwIndex));
    for (long k = 0; k < nnz; ++k) {
        a->pr[k] = pr[k];
        a->ir[k] = (mwIndex)ir[k];
    }
    for (long j = 0; j <= n; ++j) a->jc[j] = (mwIndex)jc[j];
    return a;
}
/* 1 x 1 struct with nf fields */
mxArray* mock_struct(int nf, const char** names, mxArray** vals) {
    mxArray* s = mxCreateStructMatrix(1, 1, nf, names);
    for (int k = 0; k < nf; ++k) mxSetField(s, 0, names[k], vals[k]);
    return s;
}
mxArray* mock_struct2(const char* n1, mxArray* v1, const char* n2, mxArray* v2) {
    const char* names[2] = {n1, n2};
    mxArray* s = mxCreateStructMatrix(1, 1, 2, names);
    mxSetField(s, 0, n1, v1);
    mxSetField(s, 0, n2, v2);
    return s;
}
int mock_call(int nlhs, mxArray** plhs, int nrhs, const mxArray** prhs) {
    g_err_id[0] = g_err_msg[0] = 0;
    if (setjmp(g_jmp)) return 1;
    mexFunction(nlhs, plhs, nrhs, prhs);
    return 0;
}
const char* mock_err_id(void) { return g_err_id; }
const char* mock_err_msg(void) { return g_err_msg; }
double* mock_data(const mxArray* a) { return a ? a->pr : NULL; }
size_t mock_numel(const mxArray* a) { return a ? mxGetNumberOfElements(a) : 0; }
mxArray* mock_field(const mxArray* a, const char* name) { return mxGetField(a, 0, name); }
const char* mock_string(const mxArray* a) { return a && a->str ? a->str : ""; }
void mock_atexit(void) {
    if (g_atexit) g_atexit();
    g_atexit = NULL;
}
