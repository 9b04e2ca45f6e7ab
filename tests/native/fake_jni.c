/*
 * fake_jni.c -- a test JNIEnv for java/jni/hgx_jni.c.  TEST INFRASTRUCTURE (no JDK exists in this
 * image): it lets the shim run for real, called through its exported
 * Java_org_hypergraphdb_gpu_Hgx_* symbols from the Python tests (tests/jni_harness.py) and from the
 * host sanitizer driver (tests/native/host_check.cc).
 *
 * What it models of a JVM, and checks:
 *   - Java arrays and strings are heap objects with a length (jobject = pointer to the object);
 *   - Get<T>ArrayElements hands out a COPY (isCopy = true, as a VM with a moving collector may):
 *     the shim must not rely on writes to it, and a copy released with JNI_ABORT must come back
 *     unmodified (the ABI only reads its inputs) -- a modified copy is a violation;
 *   - every pin / GetStringUTFChars must be released exactly once (outstanding pins after a native
 *     returns are a leak the harness reports);
 *   - ThrowNew records a pending exception (class + message); while one is pending, only the
 *     Release* functions may be called (JNI spec, "Exception handling"); anything else, or a second
 *     ThrowNew, is a violation;
 *   - an OutOfMemory injection makes the n-th array allocation or pin fail as a VM would (NULL +
 *     pending OutOfMemoryError).
 * Each env is independent (one per test thread).
 */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { K_INT = 0, K_LONG = 1, K_BYTE = 2, K_DOUBLE = 3, K_STRING = 4, K_CLASS = 5 };
static const size_t k_elem[] = {4, 8, 1, 8, 1, 1};

struct _jobject {
    int kind;
    int64_t n;              /* elements (strings: bytes without the terminator) */
    void *data;
    struct _jobject *next;  /* the env's object list */
    int freed;
};

typedef struct fj_pin {
    struct _jobject *obj;
    void *copy;
    struct fj_pin *next;
} fj_pin;

typedef struct fj_env {
    const struct JNINativeInterface_ *fns;   /* first member: a JNIEnv* points here */
    struct _jobject *objs;
    fj_pin *pins;
    int64_t n_pins;
    char exc_class[128];
    char exc_msg[1024];
    int exc_pending;
    int violations;
    char violation[512];
    int64_t oom_countdown;   /* > 0: the n-th allocation / pin fails */
} fj_env;

#define ENV(e) ((fj_env *)(e))

static void violate(fj_env *f, const char *what) {
    if (!f->violations) snprintf(f->violation, sizeof f->violation, "%s", what);
    f->violations++;
}
/* every JNI function except the Release* family must not run with an exception pending */
static void need_clear(fj_env *f, const char *fn) {
    if (!f->exc_pending) return;
    char m[256];
    snprintf(m, sizeof m, "%s called with a pending %s", fn, f->exc_class);
    violate(f, m);
}
static int oom_now(fj_env *f) {
    if (f->oom_countdown <= 0) return 0;
    if (--f->oom_countdown > 0) return 0;
    snprintf(f->exc_class, sizeof f->exc_class, "java/lang/OutOfMemoryError");
    snprintf(f->exc_msg, sizeof f->exc_msg, "injected");
    f->exc_pending = 1;
    return 1;
}

static struct _jobject *new_obj(fj_env *f, int kind, int64_t n) {
    struct _jobject *o = (struct _jobject *)calloc(1, sizeof *o);
    o->kind = kind;
    o->n = n;
    o->data = calloc((size_t)(n > 0 ? n : 1) + (kind == K_STRING || kind == K_CLASS), k_elem[kind]);   /* names: + NUL */
    o->next = f->objs;
    f->objs = o;
    return o;
}

static int is_array(struct _jobject *o, int kind) { return o && !o->freed && o->kind == kind; }

/* ---- the JNI functions the shim uses -------------------------------------------------------- */

static jclass fj_FindClass(JNIEnv *e, const char *name) {
    fj_env *f = ENV(e);
    need_clear(f, "FindClass");
    struct _jobject *o = new_obj(f, K_CLASS, (int64_t)strlen(name));
    memcpy(o->data, name, strlen(name) + 1);
    return (jclass)o;
}

static jint fj_ThrowNew(JNIEnv *e, jclass c, const char *msg) {
    fj_env *f = ENV(e);
    if (f->exc_pending) violate(f, "ThrowNew with an exception already pending");
    struct _jobject *o = (struct _jobject *)c;
    if (!o || o->kind != K_CLASS) { violate(f, "ThrowNew on a non-class"); return -1; }
    snprintf(f->exc_class, sizeof f->exc_class, "%s", (const char *)o->data);
    snprintf(f->exc_msg, sizeof f->exc_msg, "%s", msg ? msg : "");
    f->exc_pending = 1;
    return 0;
}

static jsize fj_GetArrayLength(JNIEnv *e, jarray a) {
    fj_env *f = ENV(e);
    need_clear(f, "GetArrayLength");
    struct _jobject *o = (struct _jobject *)a;
    if (!o || o->freed || o->kind == K_STRING || o->kind == K_CLASS) { violate(f, "GetArrayLength on a non-array"); return 0; }
    return (jsize)o->n;
}

static void *pin(JNIEnv *e, jarray a, int kind, const char *fn) {
    fj_env *f = ENV(e);
    need_clear(f, fn);
    struct _jobject *o = (struct _jobject *)a;
    if (!is_array(o, kind)) { violate(f, "Get<T>ArrayElements on an array of another type"); return NULL; }
    if (oom_now(f)) return NULL;
    fj_pin *p = (fj_pin *)calloc(1, sizeof *p);
    p->obj = o;
    p->copy = malloc((size_t)(o->n > 0 ? o->n : 1) * k_elem[kind]);
    memcpy(p->copy, o->data, (size_t)o->n * k_elem[kind]);
    p->next = f->pins;
    f->pins = p;
    f->n_pins++;
    return p->copy;
}
static jint *fj_GetIntArrayElements(JNIEnv *e, jintArray a, jboolean *c) {
    if (c) *c = 1;
    return (jint *)pin(e, a, K_INT, "GetIntArrayElements");
}
static jlong *fj_GetLongArrayElements(JNIEnv *e, jlongArray a, jboolean *c) {
    if (c) *c = 1;
    return (jlong *)pin(e, a, K_LONG, "GetLongArrayElements");
}
static jbyte *fj_GetByteArrayElements(JNIEnv *e, jbyteArray a, jboolean *c) {
    if (c) *c = 1;
    return (jbyte *)pin(e, a, K_BYTE, "GetByteArrayElements");
}

static void unpin_(JNIEnv *e, jarray a, void *elems, jint mode, int kind) {
    fj_env *f = ENV(e);   /* Release* is allowed with an exception pending */
    fj_pin **pp = &f->pins;
    while (*pp && !((*pp)->copy == elems && (*pp)->obj == (struct _jobject *)a)) pp = &(*pp)->next;
    if (!*pp) { violate(f, "Release<T>ArrayElements of elements that were not pinned"); return; }
    fj_pin *p = *pp;
    const size_t bytes = (size_t)p->obj->n * k_elem[kind];
    if (p->obj->kind != kind) violate(f, "Release<T>ArrayElements with the wrong element type");
    if (mode == JNI_ABORT) {
        if (bytes && memcmp(p->copy, p->obj->data, bytes) != 0) violate(f, "the shim modified a pinned input array");
    } else {
        memcpy(p->obj->data, p->copy, bytes);   /* 0 / JNI_COMMIT: copy back */
    }
    if (mode == 1 /* JNI_COMMIT: keep the pin */) return;
    *pp = p->next;
    free(p->copy);
    free(p);
    f->n_pins--;
}
static void fj_ReleaseIntArrayElements(JNIEnv *e, jintArray a, jint *p, jint m) { unpin_(e, a, p, m, K_INT); }
static void fj_ReleaseLongArrayElements(JNIEnv *e, jlongArray a, jlong *p, jint m) { unpin_(e, a, p, m, K_LONG); }
static void fj_ReleaseByteArrayElements(JNIEnv *e, jbyteArray a, jbyte *p, jint m) { unpin_(e, a, p, m, K_BYTE); }

static jarray new_array(JNIEnv *e, jsize n, int kind, const char *fn) {
    fj_env *f = ENV(e);
    need_clear(f, fn);
    if (n < 0) { violate(f, "New<T>Array with a negative length"); return NULL; }
    if (oom_now(f)) return NULL;
    return (jarray)new_obj(f, kind, n);
}
static jintArray fj_NewIntArray(JNIEnv *e, jsize n) { return new_array(e, n, K_INT, "NewIntArray"); }
static jlongArray fj_NewLongArray(JNIEnv *e, jsize n) { return new_array(e, n, K_LONG, "NewLongArray"); }
static jbyteArray fj_NewByteArray(JNIEnv *e, jsize n) { return new_array(e, n, K_BYTE, "NewByteArray"); }
static jarray fj_NewDoubleArray(JNIEnv *e, jsize n) { return new_array(e, n, K_DOUBLE, "NewDoubleArray"); }

static void region(JNIEnv *e, jarray a, jsize s, jsize n, void *buf, int kind, int set, const char *fn) {
    fj_env *f = ENV(e);
    need_clear(f, fn);
    struct _jobject *o = (struct _jobject *)a;
    if (!is_array(o, kind)) { violate(f, "array region on an array of another type"); return; }
    if (s < 0 || n < 0 || (int64_t)s + n > o->n) {   /* the VM throws ArrayIndexOutOfBoundsException */
        violate(f, "array region out of bounds");
        return;
    }
    char *d = (char *)o->data + (size_t)s * k_elem[kind];
    if (set) memcpy(d, buf, (size_t)n * k_elem[kind]);
    else memcpy(buf, d, (size_t)n * k_elem[kind]);
}
static void fj_SetIntArrayRegion(JNIEnv *e, jintArray a, jsize s, jsize n, const jint *b) {
    region(e, a, s, n, (void *)b, K_INT, 1, "SetIntArrayRegion");
}
static void fj_SetLongArrayRegion(JNIEnv *e, jlongArray a, jsize s, jsize n, const jlong *b) {
    region(e, a, s, n, (void *)b, K_LONG, 1, "SetLongArrayRegion");
}
static void fj_SetByteArrayRegion(JNIEnv *e, jbyteArray a, jsize s, jsize n, const jbyte *b) {
    region(e, a, s, n, (void *)b, K_BYTE, 1, "SetByteArrayRegion");
}
static void fj_SetDoubleArrayRegion(JNIEnv *e, jarray a, jsize s, jsize n, const double *b) {
    region(e, a, s, n, (void *)b, K_DOUBLE, 1, "SetDoubleArrayRegion");
}
static void fj_GetByteArrayRegion(JNIEnv *e, jbyteArray a, jsize s, jsize n, jbyte *b) {
    region(e, a, s, n, b, K_BYTE, 0, "GetByteArrayRegion");
}

static const char *fj_GetStringUTFChars(JNIEnv *e, jstring s, jboolean *c) {
    fj_env *f = ENV(e);
    need_clear(f, "GetStringUTFChars");
    struct _jobject *o = (struct _jobject *)s;
    if (!o || o->freed || o->kind != K_STRING) { violate(f, "GetStringUTFChars on a non-string"); return NULL; }
    if (c) *c = 1;
    if (oom_now(f)) return NULL;
    fj_pin *p = (fj_pin *)calloc(1, sizeof *p);
    p->obj = o;
    p->copy = malloc((size_t)o->n + 1);
    memcpy(p->copy, o->data, (size_t)o->n + 1);
    p->next = f->pins;
    f->pins = p;
    f->n_pins++;
    return (const char *)p->copy;
}
static void fj_ReleaseStringUTFChars(JNIEnv *e, jstring s, const char *chars) {
    fj_env *f = ENV(e);
    fj_pin **pp = &f->pins;
    while (*pp && !((*pp)->copy == chars && (*pp)->obj == (struct _jobject *)s)) pp = &(*pp)->next;
    if (!*pp) { violate(f, "ReleaseStringUTFChars of chars that were not obtained"); return; }
    fj_pin *p = *pp;
    *pp = p->next;
    free(p->copy);
    free(p);
    f->n_pins--;
}

static jstring fj_NewStringUTF(JNIEnv *e, const char *s) {
    fj_env *f = ENV(e);
    need_clear(f, "NewStringUTF");
    if (!s) { violate(f, "NewStringUTF(NULL)"); return NULL; }
    if (oom_now(f)) return NULL;
    struct _jobject *o = new_obj(f, K_STRING, (int64_t)strlen(s));
    memcpy(o->data, s, strlen(s) + 1);
    return (jstring)o;
}

static jboolean fj_ExceptionCheck(JNIEnv *e) { return ENV(e)->exc_pending ? 1 : 0; }   /* allowed while pending */

static const struct JNINativeInterface_ fj_table = {
    fj_FindClass,
    fj_ThrowNew,
    fj_GetArrayLength,
    fj_GetIntArrayElements,
    fj_GetLongArrayElements,
    fj_GetByteArrayElements,
    fj_ReleaseIntArrayElements,
    fj_ReleaseLongArrayElements,
    fj_ReleaseByteArrayElements,
    fj_NewIntArray,
    fj_NewLongArray,
    fj_NewByteArray,
    fj_NewDoubleArray,
    fj_SetIntArrayRegion,
    fj_SetLongArrayRegion,
    fj_SetByteArrayRegion,
    fj_SetDoubleArrayRegion,
    fj_GetByteArrayRegion,
    fj_GetStringUTFChars,
    fj_ReleaseStringUTFChars,
    fj_NewStringUTF,
    fj_ExceptionCheck,
};

/* ---- the harness side (what the tests call) -------------------------------------------------- */

JNIEnv *fj_env_new(void) {
    fj_env *f = (fj_env *)calloc(1, sizeof *f);
    f->fns = &fj_table;
    return (JNIEnv *)f;
}

void fj_env_free(JNIEnv *e) {
    fj_env *f = ENV(e);
    for (struct _jobject *o = f->objs, *n; o; o = n) {
        n = o->next;
        free(o->data);
        free(o);
    }
    for (fj_pin *p = f->pins, *n; p; p = n) {
        n = p->next;
        free(p->copy);
        free(p);
    }
    free(f);
}

/* a Java array of kind (0 int, 1 long, 2 byte, 3 double) holding a copy of n elements */
jobject fj_new_array(JNIEnv *e, int kind, const void *data, int64_t n) {
    if (kind < K_INT || kind > K_DOUBLE || n < 0) return NULL;
    struct _jobject *o = new_obj(ENV(e), kind, n);
    if (n && data) memcpy(o->data, data, (size_t)n * k_elem[kind]);
    return (jobject)o;
}
jobject fj_new_string(JNIEnv *e, const char *s) {
    struct _jobject *o = new_obj(ENV(e), K_STRING, (int64_t)strlen(s));
    memcpy(o->data, s, strlen(s) + 1);
    return (jobject)o;
}
int fj_kind(jobject o) { return o ? ((struct _jobject *)o)->kind : -1; }
int64_t fj_length(jobject o) { return o ? ((struct _jobject *)o)->n : -1; }
const void *fj_data(jobject o) { return o ? ((struct _jobject *)o)->data : NULL; }
/* the object is dead to the test (its memory stays until fj_env_free: a stale use is caught) */
void fj_release(JNIEnv *e, jobject o) {
    (void)e;
    if (o) ((struct _jobject *)o)->freed = 1;
}

const char *fj_exception_class(JNIEnv *e) { return ENV(e)->exc_pending ? ENV(e)->exc_class : NULL; }
const char *fj_exception_message(JNIEnv *e) { return ENV(e)->exc_pending ? ENV(e)->exc_msg : NULL; }
void fj_exception_clear(JNIEnv *e) { ENV(e)->exc_pending = 0; }
int64_t fj_outstanding_pins(JNIEnv *e) { return ENV(e)->n_pins; }
int fj_violations(JNIEnv *e) { return ENV(e)->violations; }
const char *fj_violation_text(JNIEnv *e) { return ENV(e)->violation; }
void fj_inject_oom(JNIEnv *e, int64_t nth) { ENV(e)->oom_countdown = nth; }
int64_t fj_live_objects(JNIEnv *e) {
    int64_t n = 0;
    for (struct _jobject *o = ENV(e)->objs; o; o = o->next) n += !o->freed && o->kind != K_CLASS;
    return n;
}
