/*
 * mex_shim.c — TEST-ONLY implementation of tests/mex_shim/mex.h plus a tiny
 * harness (t_* functions) through which tests/test_mex_gateway.py builds
 * MATLAB-like arguments with ctypes, calls mexFunction and reads the outputs.
 * mexErrMsgIdAndTxt longjmps back to t_call, which reports the error id and
 * message (as MATLAB would raise them).
 */
#include <setjmp.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mex.h"

#define MAXF 32

struct mxArray_tag {
    mxClassID cls;
    size_t m, n;
    void* data;                 /* double / int32 / char payload, column-major */
    int nf;                     /* struct fields */
    char* fname[MAXF];
    mxArray* fval[MAXF];
};

static jmp_buf g_jmp;
static int g_in_call = 0;
static char g_err_id[128], g_err_msg[1024];
static void (*g_atexit)(void) = NULL;

static size_t elsize(mxClassID c) { return c == mxDOUBLE_CLASS ? 8 : (c == mxINT32_CLASS ? 4 : 1); }

static mxArray* make(mxClassID c, size_t m, size_t n) {
    mxArray* a = calloc(1, sizeof *a);
    a->cls = c;
    a->m = m;
    a->n = n;
    if (c != mxSTRUCT_CLASS) a->data = calloc(m * n + 1, elsize(c));
    return a;
}

void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    snprintf(g_err_id, sizeof g_err_id, "%s", id);
    vsnprintf(g_err_msg, sizeof g_err_msg, fmt, ap);
    va_end(ap);
    if (g_in_call) longjmp(g_jmp, 1);
    fprintf(stderr, "mex error outside a call: %s %s\n", g_err_id, g_err_msg);
    abort();
}
int mexAtExit(void (*fn)(void)) { g_atexit = fn; return 0; }

mxArray* mxCreateDoubleMatrix(size_t m, size_t n, mxComplexity c) { (void)c; return make(mxDOUBLE_CLASS, m, n); }
mxArray* mxCreateNumericMatrix(size_t m, size_t n, mxClassID cls, mxComplexity c) { (void)c; return make(cls, m, n); }
mxArray* mxDuplicateArray(const mxArray* a) {
    mxArray* b = make(a->cls, a->m, a->n);
    if (a->data) memcpy(b->data, a->data, a->m * a->n * elsize(a->cls));
    for (int i = 0; i < a->nf; ++i) {
        b->fname[i] = strdup(a->fname[i]);
        b->fval[i] = mxDuplicateArray(a->fval[i]);
    }
    b->nf = a->nf;
    return b;
}
void mxDestroyArray(mxArray* a) {
    if (!a) return;
    for (int i = 0; i < a->nf; ++i) { free(a->fname[i]); mxDestroyArray(a->fval[i]); }
    free(a->data);
    free(a);
}
mxArray* mxGetField(const mxArray* s, size_t i, const char* name) {
    (void)i;
    if (!s || s->cls != mxSTRUCT_CLASS) return NULL;
    for (int k = 0; k < s->nf; ++k)
        if (!strcmp(s->fname[k], name)) return s->fval[k];
    return NULL;
}
int mxIsDouble(const mxArray* a) { return a && a->cls == mxDOUBLE_CLASS; }
int mxIsInt32(const mxArray* a) { return a && a->cls == mxINT32_CLASS; }
int mxIsChar(const mxArray* a) { return a && a->cls == mxCHAR_CLASS; }
int mxIsStruct(const mxArray* a) { return a && a->cls == mxSTRUCT_CLASS; }
int mxIsComplex(const mxArray* a) { (void)a; return 0; }
size_t mxGetM(const mxArray* a) { return a->m; }
size_t mxGetN(const mxArray* a) { return a->n; }
size_t mxGetNumberOfElements(const mxArray* a) { return a->cls == mxSTRUCT_CLASS ? 1 : a->m * a->n; }
double* mxGetDoubles(const mxArray* a) { return a->cls == mxDOUBLE_CLASS ? (double*)a->data : NULL; }
int32_t* mxGetInt32s(const mxArray* a) { return a->cls == mxINT32_CLASS ? (int32_t*)a->data : NULL; }
double mxGetScalar(const mxArray* a) {
    if (a->cls == mxDOUBLE_CLASS) return ((double*)a->data)[0];
    if (a->cls == mxINT32_CLASS) return ((int32_t*)a->data)[0];
    return 0.0;
}
int mxGetString(const mxArray* a, char* buf, size_t n) {
    if (a->cls != mxCHAR_CLASS || n == 0) return 1;
    snprintf(buf, n, "%s", (const char*)a->data);
    return strlen((const char*)a->data) >= n;
}

/* ---- harness ---- */
mxArray* t_double(size_t m, size_t n, const double* d) {
    mxArray* a = make(mxDOUBLE_CLASS, m, n);
    if (d) memcpy(a->data, d, m * n * 8);
    return a;
}
mxArray* t_int32(size_t m, size_t n, const int32_t* d) {
    mxArray* a = make(mxINT32_CLASS, m, n);
    if (d) memcpy(a->data, d, m * n * 4);
    return a;
}
mxArray* t_char(const char* s) {
    mxArray* a = make(mxCHAR_CLASS, 1, strlen(s));
    free(a->data);
    a->data = strdup(s);
    return a;
}
mxArray* t_struct(void) { return make(mxSTRUCT_CLASS, 1, 1); }
void t_struct_set(mxArray* s, const char* name, mxArray* v) {
    s->fname[s->nf] = strdup(name);
    s->fval[s->nf++] = v;
}
int t_class(const mxArray* a) { return (int)a->cls; }
size_t t_m(const mxArray* a) { return a->m; }
size_t t_n(const mxArray* a) { return a->n; }
void* t_data(const mxArray* a) { return a->data; }
void t_free(mxArray* a) { mxDestroyArray(a); }
const char* t_err_id(void) { return g_err_id; }
const char* t_err_msg(void) { return g_err_msg; }
/* call mexFunction; 0 = returned, 1 = raised (t_err_id / t_err_msg) */
int t_call(int nlhs, mxArray** plhs, int nrhs, mxArray** prhs) {
    g_err_id[0] = g_err_msg[0] = 0;
    g_in_call = 1;
    if (setjmp(g_jmp)) {
        g_in_call = 0;
        return 1;
    }
    for (int i = 0; i < nlhs; ++i) plhs[i] = NULL;
    mexFunction(nlhs, plhs, nrhs, (const mxArray**)prhs);
    g_in_call = 0;
    return 0;
}
/* what MATLAB does on `clear mex`: the gateway's mexAtExit handler */
int t_clear(void) {
    if (!g_atexit) return 0;
    g_atexit();
    g_atexit = NULL;
    return 1;
}
