/*
 * hgx_jni.c -- JNI shim between org.hypergraphdb.gpu.Hgx (java/org/hypergraphdb/gpu/Hgx.java) and
 * the C ABI of libhgx.so (include/hgx.h).  Arrays in, handles (jlong) out; a nonzero status becomes
 * an exception: HGX_E_UNSUPPORTED -> java.lang.UnsupportedOperationException (the Java caller keeps
 * the reference class), HGX_E_NOMEM -> OutOfMemoryError, anything else -> org.hypergraphdb.HGException
 * with hgx_last_error().  Arguments the shim itself rejects (inconsistent array lengths, offset tables
 * that would reach past their data array) throw java.lang.IllegalArgumentException with the shim's own
 * message, before the engine is called: the C ABI cannot see Java array lengths and would read past
 * the pinned array.  A result too large for one Java array throws UnsupportedOperationException.
 * Primitive arrays are pinned with Get<T>ArrayElements and released with JNI_ABORT (the ABI
 * deep-copies every input); no pointer into the JVM heap outlives a call, and nothing calls back
 * into the JVM (ownership).
 *
 * Build (a host with a JDK):
 *   gcc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *       java/jni/hgx_jni.c -Lhypergraphdb_amd -lhgx -Wl,-rpath,'$ORIGIN' -o libhgx_jni.so
 *
 * No JDK exists in this build image.  The shim is executed instead through a
 * test JNIEnv (tests/native/fake_jni.c: arrays as heap objects, copy-mode pinning, exceptions
 * recorded, JNI-call discipline checked) -- tests/test_jni.py drives every native on the CPU and
 * tests/test_gpu_jni.py on the GPU against the oracle.
 */
#include <jni.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hgx.h"

#define JFN(name) JNICALL Java_org_hypergraphdb_gpu_Hgx_##name

/* the largest element count of one Java array (VMs reserve a few header words below INT_MAX) */
#define HGX_JARRAY_MAX ((int64_t)0x7fffffff - 8)

static void throw_class(JNIEnv *e, const char *cls, const char *msg) {
    jclass c = (*e)->FindClass(e, cls);
    if (c) (*e)->ThrowNew(e, c, msg);
}

static void throw_rc(JNIEnv *e, int rc) {
    throw_class(e, rc == HGX_E_UNSUPPORTED ? "java/lang/UnsupportedOperationException"
                   : rc == HGX_E_NOMEM     ? "java/lang/OutOfMemoryError"
                                           : "org/hypergraphdb/HGException",
                hgx_last_error());
}

static void throw_msg(JNIEnv *e, const char *msg) { throw_class(e, "java/lang/IllegalArgumentException", msg); }

/* A result of n elements must fit one Java array. */
static int fits_jarray(JNIEnv *e, int64_t n, const char *what) {
    if (n >= 0 && n <= HGX_JARRAY_MAX) return 1;
    char m[160];
    snprintf(m, sizeof m, "%s: %lld elements do not fit one Java array", what, (long long)n);
    throw_class(e, "java/lang/UnsupportedOperationException", m);
    return 0;
}

/* Pinned views of Java arrays (NULL array -> NULL pointer, length 0).  A pin after a failed one
 * (OutOfMemoryError pending) is skipped: no JNI call but Release* may run with an exception pending. */
typedef struct { jarray a; void *p; jsize n; int kind; } pin_t;   /* kind: 0 int, 1 long, 2 byte */

static pin_t pin_int(JNIEnv *e, jintArray a) {
    pin_t r = {a, NULL, 0, 0};
    if (a && !(*e)->ExceptionCheck(e)) { r.n = (*e)->GetArrayLength(e, a); r.p = (*e)->GetIntArrayElements(e, a, NULL); }
    return r;
}
static pin_t pin_long(JNIEnv *e, jlongArray a) {
    pin_t r = {a, NULL, 0, 1};
    if (a && !(*e)->ExceptionCheck(e)) { r.n = (*e)->GetArrayLength(e, a); r.p = (*e)->GetLongArrayElements(e, a, NULL); }
    return r;
}
static pin_t pin_byte(JNIEnv *e, jbyteArray a) {
    pin_t r = {a, NULL, 0, 2};
    if (a && !(*e)->ExceptionCheck(e)) { r.n = (*e)->GetArrayLength(e, a); r.p = (*e)->GetByteArrayElements(e, a, NULL); }
    return r;
}
static void unpin(JNIEnv *e, pin_t *x) {
    if (!x->a || !x->p) return;
    if (x->kind == 0) (*e)->ReleaseIntArrayElements(e, (jintArray)x->a, (jint *)x->p, JNI_ABORT);
    else if (x->kind == 1) (*e)->ReleaseLongArrayElements(e, (jlongArray)x->a, (jlong *)x->p, JNI_ABORT);
    else (*e)->ReleaseByteArrayElements(e, (jbyteArray)x->a, (jbyte *)x->p, JNI_ABORT);
    x->p = NULL;
}
/* an output array: its elements are copied back into the Java array (mode 0) */
static void unpin_out(JNIEnv *e, pin_t *x) {
    if (!x->a || !x->p) return;
    if (x->kind == 0) (*e)->ReleaseIntArrayElements(e, (jintArray)x->a, (jint *)x->p, 0);
    else if (x->kind == 1) (*e)->ReleaseLongArrayElements(e, (jlongArray)x->a, (jlong *)x->p, 0);
    else (*e)->ReleaseByteArrayElements(e, (jbyteArray)x->a, (jbyte *)x->p, 0);
    x->p = NULL;
}
/* a pin of a non-null array whose elements could not be obtained (the VM has thrown OutOfMemoryError) */
static int pin_failed(const pin_t *x) { return x->a && !x->p; }

/* ---- argument checks (each throws IllegalArgumentException and returns 0 on failure) ----------- */

static int check_len(JNIEnv *e, const pin_t *x, int64_t want, const char *name) {
    if (pin_failed(x)) return 0;   /* OutOfMemoryError already pending */
    if ((int64_t)x->n == want) return 1;
    char m[200];
    snprintf(m, sizeof m, "%s: length %lld, expected %lld", name, (long long)x->n, (long long)want);
    throw_msg(e, m);
    return 0;
}

/* An offsets table of n1 entries into a data array of data_len elements (stride elements per offset
 * unit): off[0] = 0, never decreasing, off[n1-1] * stride <= data_len.  Every slice the engine reads
 * then lies inside the pinned data array. */
static int check_offsets(JNIEnv *e, const pin_t *off, int64_t n1, int64_t data_len, int64_t stride,
                         const char *name) {
    if (!check_len(e, off, n1, name)) return 0;
    const int64_t *o = (const int64_t *)off->p;
    char m[200];
    if (n1 == 0) return 1;
    if (!o) { snprintf(m, sizeof m, "%s: null", name); throw_msg(e, m); return 0; }
    if (o[0] != 0) {
        snprintf(m, sizeof m, "%s[0] = %lld, expected 0", name, (long long)o[0]);
        throw_msg(e, m);
        return 0;
    }
    for (int64_t i = 1; i < n1; i++)
        if (o[i] < o[i - 1]) {
            snprintf(m, sizeof m, "%s decreases at index %lld", name, (long long)i);
            throw_msg(e, m);
            return 0;
        }
    if (o[n1 - 1] > data_len / stride) {
        snprintf(m, sizeof m, "%s ends at %lld, beyond its data array (%lld elements)", name, (long long)o[n1 - 1],
                 (long long)data_len);
        throw_msg(e, m);
        return 0;
    }
    return 1;
}

static int check_not_null(JNIEnv *e, const void *p, const char *name) {
    if (p) return 1;
    char m[120];
    snprintf(m, sizeof m, "%s is null", name);
    throw_class(e, "java/lang/NullPointerException", m);
    return 0;
}

static jintArray new_ints(JNIEnv *e, const int32_t *v, int64_t n) {
    if (!fits_jarray(e, n, "int[] result")) return NULL;
    jintArray a = (*e)->NewIntArray(e, (jsize)n);
    if (a && n) (*e)->SetIntArrayRegion(e, a, 0, (jsize)n, (const jint *)v);
    return a;
}
static jlongArray new_longs(JNIEnv *e, const int64_t *v, int64_t n) {
    if (!fits_jarray(e, n, "long[] result")) return NULL;
    jlongArray a = (*e)->NewLongArray(e, (jsize)n);
    if (a && n) (*e)->SetLongArrayRegion(e, a, 0, (jsize)n, (const jlong *)v);
    return a;
}

static hgx_graph_desc desc_of(jlong numAtoms, pin_t *la, pin_t *off, pin_t *tg, pin_t *ty) {
    hgx_graph_desc d;
    d.num_atoms = numAtoms;
    d.num_links = la->n;
    d.link_atom = (const int32_t *)la->p;
    d.tgt_off = (const int64_t *)off->p;
    d.tgt_idx = (const int32_t *)tg->p;
    d.link_type = (const int32_t *)ty->p;
    return d;
}

/* The snapshot rows of hgx_graph_desc: tgtOff has M+1 entries ending within tgtIdx, linkType is null
 * or has M entries. */
static int check_rows(JNIEnv *e, const pin_t *la, const pin_t *off, const pin_t *tg, const pin_t *ty) {
    if (pin_failed(la) || pin_failed(tg)) return 0;
    return check_offsets(e, off, (int64_t)la->n + 1, tg->n, 1, "tgtOff") &&
           (!ty->a || check_len(e, ty, la->n, "linkType"));
}

/* ---- snapshot ------------------------------------------------------------------------------ */

JNIEXPORT jlong JFN(graphCreate)(JNIEnv *e, jclass k, jlong numAtoms, jintArray linkAtom, jlongArray tgtOff,
                                 jintArray tgtIdx, jintArray linkType, jint device) {
    pin_t la = pin_int(e, linkAtom), off = pin_long(e, tgtOff), tg = pin_int(e, tgtIdx), ty = pin_int(e, linkType);
    hgx_graph *g = NULL;
    int ok = check_rows(e, &la, &off, &tg, &ty), rc = HGX_OK;
    if (ok) {
        hgx_graph_desc d = desc_of(numAtoms, &la, &off, &tg, &ty);
        rc = hgx_graph_create(&d, device, &g);
    }
    unpin(e, &la); unpin(e, &off); unpin(e, &tg); unpin(e, &ty);
    if (ok && rc) throw_rc(e, rc);
    return ok && !rc ? (jlong)(intptr_t)g : 0;
}

JNIEXPORT jlong JFN(graphOpen)(JNIEnv *e, jclass k, jstring path, jint device) {
    if (!check_not_null(e, path, "path")) return 0;
    const char *p = (*e)->GetStringUTFChars(e, path, NULL);
    if (!p) return 0;
    hgx_graph *g = NULL;
    int rc = hgx_graph_open(p, device, &g);
    (*e)->ReleaseStringUTFChars(e, path, p);
    if (rc) { throw_rc(e, rc); return 0; }
    return (jlong)(intptr_t)g;
}

JNIEXPORT void JFN(graphDestroy)(JNIEnv *e, jclass k, jlong g) { hgx_graph_destroy((hgx_graph *)(intptr_t)g); }

JNIEXPORT jlong JFN(graphContext)(JNIEnv *e, jclass k, jlong g) {
    hgx_graph *c = NULL;
    int rc = hgx_graph_context((hgx_graph *)(intptr_t)g, &c);
    if (rc) { throw_rc(e, rc); return 0; }
    return (jlong)(intptr_t)c;
}

JNIEXPORT jlongArray JFN(graphInfo)(JNIEnv *e, jclass k, jlong g) {
    int64_t v[3];
    int rc = hgx_graph_info((hgx_graph *)(intptr_t)g, &v[0], &v[1], &v[2]);
    if (rc) { throw_rc(e, rc); return NULL; }
    return new_longs(e, v, 3);
}

JNIEXPORT void JFN(graphUpdate)(JNIEnv *e, jclass k, jlong g, jlong numAtoms, jintArray addLinkAtom,
                                jlongArray addTgtOff, jintArray addTgtIdx, jintArray addLinkType,
                                jintArray removeLinkAtom) {
    pin_t la = pin_int(e, addLinkAtom), off = pin_long(e, addTgtOff), tg = pin_int(e, addTgtIdx),
          ty = pin_int(e, addLinkType), rm = pin_int(e, removeLinkAtom);
    /* no additions: addTgtOff may be null or {0} */
    int ok = !pin_failed(&rm) && (la.n == 0 && off.n <= 1 ? (off.n == 0 || check_offsets(e, &off, 1, tg.n, 1, "addTgtOff"))
                                                         : check_rows(e, &la, &off, &tg, &ty));
    int rc = HGX_OK;
    if (ok)
        rc = hgx_graph_update((hgx_graph *)(intptr_t)g, numAtoms, la.n, (const int32_t *)la.p, (const int64_t *)off.p,
                              (const int32_t *)tg.p, (const int32_t *)ty.p, rm.n, (const int32_t *)rm.p);
    unpin(e, &la); unpin(e, &off); unpin(e, &tg); unpin(e, &ty); unpin(e, &rm);
    if (ok && rc) throw_rc(e, rc);
}

JNIEXPORT jintArray JFN(incidence)(JNIEnv *e, jclass k, jlong g, jint atom) {
    int64_t n = 0;
    int rc = hgx_graph_incidence((hgx_graph *)(intptr_t)g, atom, NULL, 0, &n);
    if (rc) { throw_rc(e, rc); return NULL; }
    if (!fits_jarray(e, n, "incidence")) return NULL;
    int32_t *buf = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    if (!buf) { throw_class(e, "java/lang/OutOfMemoryError", "incidence buffer"); return NULL; }
    rc = hgx_graph_incidence((hgx_graph *)(intptr_t)g, atom, buf, n, &n);
    jintArray out = rc ? NULL : new_ints(e, buf, n);
    free(buf);
    if (rc) throw_rc(e, rc);
    return out;
}

JNIEXPORT jlongArray JFN(degree)(JNIEnv *e, jclass k, jlong g, jintArray atoms) {
    pin_t a = pin_int(e, atoms);
    if (pin_failed(&a)) return NULL;
    int64_t *deg = (int64_t *)malloc(sizeof(int64_t) * (size_t)(a.n > 0 ? a.n : 1));
    int rc = deg ? hgx_graph_degree((hgx_graph *)(intptr_t)g, (const int32_t *)a.p, a.n, deg) : HGX_E_NOMEM;
    jlongArray out = rc ? NULL : new_longs(e, deg, a.n);
    unpin(e, &a);
    free(deg);
    if (rc) throw_rc(e, rc);
    return out;
}

JNIEXPORT void JFN(setOption)(JNIEnv *e, jclass k, jlong g, jint option, jlong value) {
    int rc = hgx_set_option((hgx_graph *)(intptr_t)g, option, value);
    if (rc) throw_rc(e, rc);
}

JNIEXPORT void JFN(snapshotWrite)(JNIEnv *e, jclass k, jstring path, jlong numAtoms, jintArray linkAtom,
                                  jlongArray tgtOff, jintArray tgtIdx, jintArray linkType, jbyteArray handles,
                                  jint handleBytes) {
    if (!check_not_null(e, path, "path")) return;
    pin_t la = pin_int(e, linkAtom), off = pin_long(e, tgtOff), tg = pin_int(e, tgtIdx), ty = pin_int(e, linkType),
          hb = pin_byte(e, handles);
    int ok = check_rows(e, &la, &off, &tg, &ty) && !pin_failed(&hb), rc = HGX_OK;
    if (ok && hb.a && (handleBytes <= 0 || numAtoms < 0 || (int64_t)hb.n != numAtoms * (int64_t)handleBytes)) {
        char m[200];
        snprintf(m, sizeof m, "handles: length %lld, expected numAtoms * handleBytes = %lld", (long long)hb.n,
                 (long long)numAtoms * (long long)handleBytes);
        throw_msg(e, m);
        ok = 0;
    }
    const char *p = ok ? (*e)->GetStringUTFChars(e, path, NULL) : NULL;
    if (ok && !p) ok = 0;
    if (ok) {
        hgx_graph_desc d = desc_of(numAtoms, &la, &off, &tg, &ty);
        rc = hgx_snapshot_write(p, &d, (const uint8_t *)hb.p, hb.p ? handleBytes : 0);
        (*e)->ReleaseStringUTFChars(e, path, p);
    }
    unpin(e, &la); unpin(e, &off); unpin(e, &tg); unpin(e, &ty); unpin(e, &hb);
    if (ok && rc) throw_rc(e, rc);
}

JNIEXPORT jlongArray JFN(snapshotInfo)(JNIEnv *e, jclass k, jstring path) {
    if (!check_not_null(e, path, "path")) return NULL;
    const char *p = (*e)->GetStringUTFChars(e, path, NULL);
    if (!p) return NULL;
    int64_t v[5] = {0, 0, 0, 0, 0};
    int32_t hb = 0, ht = 0;
    int rc = hgx_snapshot_info(p, &v[0], &v[1], &v[2], &hb, &ht);
    (*e)->ReleaseStringUTFChars(e, path, p);
    if (rc) { throw_rc(e, rc); return NULL; }
    v[3] = hb;
    v[4] = ht;
    return new_longs(e, v, 5);
}

JNIEXPORT jbyteArray JFN(snapshotHandles)(JNIEnv *e, jclass k, jstring path) {
    if (!check_not_null(e, path, "path")) return NULL;
    const char *p = (*e)->GetStringUTFChars(e, path, NULL);
    if (!p) return NULL;
    int64_t A = 0;
    int32_t hb = 0;
    int rc = hgx_snapshot_info(p, &A, NULL, NULL, &hb, NULL);
    jbyteArray out = NULL;
    int thrown = 0;
    if (!rc && hb > 0) {
        const int64_t bytes = A * (int64_t)hb;
        if (!fits_jarray(e, bytes, "snapshot handle table")) {
            thrown = 1;
        } else {
            uint8_t *buf = (uint8_t *)malloc((size_t)(bytes > 0 ? bytes : 1));
            rc = buf ? hgx_snapshot_read(p, NULL, NULL, NULL, NULL, buf) : HGX_E_NOMEM;
            if (!rc) {
                out = (*e)->NewByteArray(e, (jsize)bytes);
                if (out && bytes) (*e)->SetByteArrayRegion(e, out, 0, (jsize)bytes, (const jbyte *)buf);
            }
            free(buf);
        }
    }
    (*e)->ReleaseStringUTFChars(e, path, p);
    if (rc && !thrown) throw_rc(e, rc);
    return out;
}

/* The file's checksum over every section (hgx_snapshot_read with no outputs maps and verifies). */
JNIEXPORT void JFN(snapshotVerify)(JNIEnv *e, jclass k, jstring path) {
    if (!check_not_null(e, path, "path")) return;
    const char *p = (*e)->GetStringUTFChars(e, path, NULL);
    if (!p) return;
    int rc = hgx_snapshot_read(p, NULL, NULL, NULL, NULL, NULL);
    (*e)->ReleaseStringUTFChars(e, path, p);
    if (rc) throw_rc(e, rc);
}

/* Handles of ranks [first, first + n) (n * handle_bytes bytes): the reader of tables beyond one Java
 * array (300M 16-byte handles = 4.8 GB); the caller verifies the file once with snapshotVerify. */
JNIEXPORT jbyteArray JFN(snapshotHandlesRange)(JNIEnv *e, jclass k, jstring path, jlong first, jlong n) {
    if (!check_not_null(e, path, "path")) return NULL;
    if (first < 0 || n < 0) { throw_msg(e, "snapshotHandlesRange: negative first or n"); return NULL; }
    const char *p = (*e)->GetStringUTFChars(e, path, NULL);
    if (!p) return NULL;
    int64_t A = 0;
    int32_t hb = 0;
    int rc = hgx_snapshot_info(p, &A, NULL, NULL, &hb, NULL), thrown = 0;
    jbyteArray out = NULL;
    if (!rc && hb <= 0) rc = HGX_E_NOTFOUND;
    if (!rc && (first > A || n > A - first)) {
        char m[200];
        snprintf(m, sizeof m, "snapshotHandlesRange: ranks [%lld, %lld) outside [0, %lld)", (long long)first,
                 (long long)(first + n), (long long)A);
        throw_msg(e, m);
        thrown = 1;
    }
    if (!rc && !thrown) {
        const int64_t bytes = n * (int64_t)hb;
        if (!fits_jarray(e, bytes, "snapshot handle range")) {
            thrown = 1;
        } else {
            uint8_t *buf = (uint8_t *)malloc((size_t)(bytes > 0 ? bytes : 1));
            rc = buf ? hgx_snapshot_read_handles(p, first, n, 0, buf) : HGX_E_NOMEM;
            if (!rc) {
                out = (*e)->NewByteArray(e, (jsize)bytes);
                if (out && bytes) (*e)->SetByteArrayRegion(e, out, 0, (jsize)bytes, (const jbyte *)buf);
            }
            free(buf);
        }
    }
    (*e)->ReleaseStringUTFChars(e, path, p);
    if (rc && !thrown) throw_rc(e, rc);
    return out;
}

/* Streaming writer (hgx_snapshot_writer_*): the rows at begin, the handle table in pieces of whole
 * handles, end = checksum + atomic replace.  The exporter of a store larger than one Java array. */
JNIEXPORT jlong JFN(snapshotWriterBegin)(JNIEnv *e, jclass k, jstring path, jlong numAtoms, jintArray linkAtom,
                                         jlongArray tgtOff, jintArray tgtIdx, jintArray linkType, jint handleBytes) {
    if (!check_not_null(e, path, "path")) return 0;
    pin_t la = pin_int(e, linkAtom), off = pin_long(e, tgtOff), tg = pin_int(e, tgtIdx), ty = pin_int(e, linkType);
    int ok = check_rows(e, &la, &off, &tg, &ty), rc = HGX_OK;
    hgx_snapshot_writer *w = NULL;
    const char *p = ok ? (*e)->GetStringUTFChars(e, path, NULL) : NULL;
    if (ok && !p) ok = 0;
    if (ok) {
        hgx_graph_desc d = desc_of(numAtoms, &la, &off, &tg, &ty);
        rc = hgx_snapshot_writer_begin(p, &d, handleBytes, &w);
        (*e)->ReleaseStringUTFChars(e, path, p);
    }
    unpin(e, &la); unpin(e, &off); unpin(e, &tg); unpin(e, &ty);
    if (ok && rc) throw_rc(e, rc);
    return ok && !rc ? (jlong)(intptr_t)w : 0;
}

/* handles.length must be a whole number of handles (checked by the engine against num_atoms). */
JNIEXPORT void JFN(snapshotWriterHandles)(JNIEnv *e, jclass k, jlong w, jbyteArray handles, jint handleBytes) {
    if (!check_not_null(e, handles, "handles")) return;
    if (handleBytes <= 0) { throw_msg(e, "snapshotWriterHandles: handleBytes <= 0"); return; }
    pin_t hb = pin_byte(e, handles);
    if (pin_failed(&hb)) return;
    int rc = HGX_OK, ok = 1;
    int32_t width = 0;   /* the writer's own width sizes the read, not the caller's */
    rc = hgx_snapshot_writer_handle_bytes((const hgx_snapshot_writer *)(intptr_t)w, &width);
    if (rc) {
        unpin(e, &hb);
        throw_rc(e, rc);
        return;
    }
    if (width != handleBytes) {
        throw_msg(e, "snapshotWriterHandles: handleBytes differs from the writer's handle width");
        ok = 0;
    }
    if (ok && hb.n % width) {
        throw_msg(e, "snapshotWriterHandles: not a whole number of handles");
        ok = 0;
    }
    if (ok) rc = hgx_snapshot_writer_handles((hgx_snapshot_writer *)(intptr_t)w, (const uint8_t *)hb.p,
                                             (int64_t)hb.n / width);
    unpin(e, &hb);
    if (ok && rc) throw_rc(e, rc);
}

JNIEXPORT void JFN(snapshotWriterEnd)(JNIEnv *e, jclass k, jlong w) {
    int rc = hgx_snapshot_writer_end((hgx_snapshot_writer *)(intptr_t)w);
    if (rc) throw_rc(e, rc);
}

JNIEXPORT void JFN(snapshotWriterAbort)(JNIEnv *e, jclass k, jlong w) {
    hgx_snapshot_writer_abort((hgx_snapshot_writer *)(intptr_t)w);
}

/* ---- batched BFS ----------------------------------------------------------------------------- */

static hgx_algen_opts opts_of(jint linkType, jboolean p, jboolean s, jboolean r, jboolean src) {
    hgx_algen_opts o;
    o.link_type = linkType;
    o.return_preceding = p ? 1 : 0;
    o.return_succeeding = s ? 1 : 0;
    o.reverse_order = r ? 1 : 0;
    o.return_source = src ? 1 : 0;
    return o;
}

JNIEXPORT jlong JFN(bfsBatch)(JNIEnv *e, jclass k, jlong g, jintArray seeds, jint maxDepth, jint linkType,
                              jboolean p, jboolean s, jboolean r, jboolean src) {
    pin_t sd = pin_int(e, seeds);
    if (pin_failed(&sd)) return 0;
    hgx_algen_opts o = opts_of(linkType, p, s, r, src);
    hgx_bfs_result *res = NULL;
    int rc = hgx_bfs_batch((hgx_graph *)(intptr_t)g, (const int32_t *)sd.p, sd.n, maxDepth, &o, &res);
    unpin(e, &sd);
    if (rc) { throw_rc(e, rc); return 0; }
    return (jlong)(intptr_t)res;
}

JNIEXPORT jintArray JFN(bfsInfo)(JNIEnv *e, jclass k, jlong r) {
    int32_t v[2];
    int rc = hgx_bfs_result_info((const hgx_bfs_result *)(intptr_t)r, &v[0], &v[1]);
    if (rc) { throw_rc(e, rc); return NULL; }
    return new_ints(e, v, 2);
}

JNIEXPORT jlongArray JFN(bfsCounts)(JNIEnv *e, jclass k, jlong r) {
    int32_t ns = 0, nl = 0;
    int rc = hgx_bfs_result_info((const hgx_bfs_result *)(intptr_t)r, &ns, &nl);
    if (rc) { throw_rc(e, rc); return NULL; }
    const int64_t n = (int64_t)ns * nl;
    if (!fits_jarray(e, n, "bfsCounts")) return NULL;
    int64_t *c = (int64_t *)malloc(sizeof(int64_t) * ((size_t)n + 1));
    rc = c ? hgx_bfs_result_counts((hgx_bfs_result *)(intptr_t)r, c) : HGX_E_NOMEM;
    jlongArray out = rc ? NULL : new_longs(e, c, n);
    free(c);
    if (rc) throw_rc(e, rc);
    return out;
}

JNIEXPORT jintArray JFN(bfsVisited)(JNIEnv *e, jclass k, jlong r, jint seedIndex, jint depth) {
    int64_t n = 0;
    hgx_bfs_result *res = (hgx_bfs_result *)(intptr_t)r;
    int rc = hgx_bfs_result_visited(res, seedIndex, depth, NULL, 0, &n);
    if (rc) { throw_rc(e, rc); return NULL; }
    if (!fits_jarray(e, n, "bfsVisited")) return NULL;
    int32_t *buf = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    rc = buf ? hgx_bfs_result_visited(res, seedIndex, depth, buf, n, &n) : HGX_E_NOMEM;
    jintArray out = rc ? NULL : new_ints(e, buf, n);
    free(buf);
    if (rc) throw_rc(e, rc);
    return out;
}

/* V_d[first, first + max) of seed seedIndex: the paged reader of sets beyond one Java array. */
JNIEXPORT jintArray JFN(bfsVisitedRange)(JNIEnv *e, jclass k, jlong r, jint seedIndex, jint depth, jlong first,
                                         jint max) {
    if (first < 0 || max < 0) { throw_msg(e, "bfsVisitedRange: negative first or max"); return NULL; }
    int32_t *buf = (int32_t *)malloc(sizeof(int32_t) * (size_t)(max > 0 ? max : 1));
    if (!buf) { throw_class(e, "java/lang/OutOfMemoryError", "visited page"); return NULL; }
    int64_t n = 0;
    int rc = hgx_bfs_result_visited_range((hgx_bfs_result *)(intptr_t)r, seedIndex, depth, first, buf, max, &n);
    const int64_t got = n > first ? (n - first < max ? n - first : max) : 0;
    jintArray out = rc ? NULL : new_ints(e, buf, got);
    free(buf);
    if (rc) throw_rc(e, rc);
    return out;
}

JNIEXPORT jint JFN(bfsDepthOf)(JNIEnv *e, jclass k, jlong r, jint seedIndex, jint atom) {
    int32_t d = -1;
    int rc = hgx_bfs_result_depth_of((hgx_bfs_result *)(intptr_t)r, seedIndex, atom, &d);
    if (rc) throw_rc(e, rc);
    return d;
}

JNIEXPORT void JFN(bfsFree)(JNIEnv *e, jclass k, jlong r) { hgx_bfs_result_free((hgx_bfs_result *)(intptr_t)r); }

/* ---- order-exact traversal ------------------------------------------------------------------- */

JNIEXPORT jlong JFN(bfsSequence)(JNIEnv *e, jclass k, jlong g, jintArray seeds, jint maxDepth, jint linkType,
                                 jboolean p, jboolean s, jboolean r, jboolean src) {
    pin_t sd = pin_int(e, seeds);
    if (pin_failed(&sd)) return 0;
    hgx_algen_opts o = opts_of(linkType, p, s, r, src);
    hgx_seq_result *res = NULL;
    int rc = hgx_bfs_sequence((hgx_graph *)(intptr_t)g, (const int32_t *)sd.p, sd.n, maxDepth, &o, &res);
    unpin(e, &sd);
    if (rc) { throw_rc(e, rc); return 0; }
    return (jlong)(intptr_t)res;
}

JNIEXPORT jlongArray JFN(seqOffsets)(JNIEnv *e, jclass k, jlong sq) {
    const hgx_seq_result *s = (const hgx_seq_result *)(intptr_t)sq;
    int32_t ns = 0, nl = 0;
    int64_t np = 0;
    int rc = hgx_seq_result_info(s, &ns, &np, &nl);
    if (rc) { throw_rc(e, rc); return NULL; }
    int64_t *off = (int64_t *)malloc(sizeof(int64_t) * ((size_t)ns + 1));
    rc = off ? hgx_seq_result_offsets(s, off) : HGX_E_NOMEM;
    jlongArray out = rc ? NULL : new_longs(e, off, (int64_t)ns + 1);
    free(off);
    if (rc) throw_rc(e, rc);
    return out;
}

/* which: 0 links, 1 atoms, 2 distances */
static jintArray seq_column(JNIEnv *e, jlong sq, int which) {
    const hgx_seq_result *s = (const hgx_seq_result *)(intptr_t)sq;
    int32_t ns = 0, nl = 0;
    int64_t np = 0;
    int rc = hgx_seq_result_info(s, &ns, &np, &nl);
    if (rc) { throw_rc(e, rc); return NULL; }
    if (!fits_jarray(e, np, "sequence pairs")) return NULL;
    int32_t *buf = (int32_t *)malloc(sizeof(int32_t) * (size_t)(np > 0 ? np : 1));
    if (!buf) { throw_class(e, "java/lang/OutOfMemoryError", "sequence buffer"); return NULL; }
    rc = hgx_seq_result_pairs(s, which == 0 ? buf : NULL, which == 1 ? buf : NULL, which == 2 ? buf : NULL);
    jintArray out = rc ? NULL : new_ints(e, buf, np);
    free(buf);
    if (rc) throw_rc(e, rc);
    return out;
}

JNIEXPORT jintArray JFN(seqLinks)(JNIEnv *e, jclass k, jlong s) { return seq_column(e, s, 0); }
JNIEXPORT jintArray JFN(seqAtoms)(JNIEnv *e, jclass k, jlong s) { return seq_column(e, s, 1); }
JNIEXPORT jintArray JFN(seqDists)(JNIEnv *e, jclass k, jlong s) { return seq_column(e, s, 2); }
JNIEXPORT void JFN(seqFree)(JNIEnv *e, jclass k, jlong s) { hgx_seq_result_free((hgx_seq_result *)(intptr_t)s); }

/* Pairs [first, first + max) of one column (0 links, 1 atoms, 2 distances): the paged reader of
 * sequences beyond one Java array. */
JNIEXPORT jintArray JFN(seqRange)(JNIEnv *e, jclass k, jlong sq, jint which, jlong first, jint max) {
    if (first < 0 || max < 0 || which < 0 || which > 2) { throw_msg(e, "seqRange: bad argument"); return NULL; }
    int32_t *buf = (int32_t *)malloc(sizeof(int32_t) * (size_t)(max > 0 ? max : 1));
    if (!buf) { throw_class(e, "java/lang/OutOfMemoryError", "sequence page"); return NULL; }
    int64_t got = 0;
    int rc = hgx_seq_result_pairs_range((const hgx_seq_result *)(intptr_t)sq, first, max, which == 0 ? buf : NULL,
                                        which == 1 ? buf : NULL, which == 2 ? buf : NULL, &got);
    jintArray out = rc ? NULL : new_ints(e, buf, got);
    free(buf);
    if (rc) throw_rc(e, rc);
    return out;
}

/* ---- conjunctive pattern batches ------------------------------------------------------------- */

/* The packed batch: n = type.length queries, incOff / patOff of n+1 entries into inc / pat,
 * hasOrdered of n entries. */
static int check_packed(JNIEnv *e, const pin_t *ty, const pin_t *io, const pin_t *ic, const pin_t *ho,
                        const pin_t *po, const pin_t *pt) {
    if (pin_failed(ty) || pin_failed(ic) || pin_failed(pt)) return 0;
    return check_offsets(e, io, (int64_t)ty->n + 1, ic->n, 1, "incOff") && check_len(e, ho, ty->n, "hasOrdered") &&
           check_offsets(e, po, (int64_t)ty->n + 1, pt->n, 1, "patOff");
}

JNIEXPORT jlong JFN(patternBatch)(JNIEnv *e, jclass k, jlong g, jintArray type, jlongArray incOff, jintArray inc,
                                  jintArray hasOrdered, jlongArray patOff, jintArray pat) {
    pin_t ty = pin_int(e, type), io = pin_long(e, incOff), ic = pin_int(e, inc), ho = pin_int(e, hasOrdered),
          po = pin_long(e, patOff), pt = pin_int(e, pat);
    hgx_query_result *q = NULL;
    int ok = check_packed(e, &ty, &io, &ic, &ho, &po, &pt), rc = HGX_OK;
    if (ok)
        rc = hgx_pattern_batch_packed((hgx_graph *)(intptr_t)g, ty.n, (const int32_t *)ty.p, (const int64_t *)io.p,
                                      (const int32_t *)ic.p, (const int32_t *)ho.p, (const int64_t *)po.p,
                                      (const int32_t *)pt.p, &q);
    unpin(e, &ty); unpin(e, &io); unpin(e, &ic); unpin(e, &ho); unpin(e, &po); unpin(e, &pt);
    if (ok && rc) throw_rc(e, rc);
    return ok && !rc ? (jlong)(intptr_t)q : 0;
}

JNIEXPORT jlong JFN(querySetCreate)(JNIEnv *e, jclass k, jlong g, jintArray type, jlongArray incOff, jintArray inc,
                                    jintArray hasOrdered, jlongArray patOff, jintArray pat) {
    pin_t ty = pin_int(e, type), io = pin_long(e, incOff), ic = pin_int(e, inc), ho = pin_int(e, hasOrdered),
          po = pin_long(e, patOff), pt = pin_int(e, pat);
    hgx_query_set *qs = NULL;
    int ok = check_packed(e, &ty, &io, &ic, &ho, &po, &pt), rc = HGX_OK;
    if (ok)
        rc = hgx_query_set_create((hgx_graph *)(intptr_t)g, ty.n, (const int32_t *)ty.p, (const int64_t *)io.p,
                                  (const int32_t *)ic.p, (const int32_t *)ho.p, (const int64_t *)po.p,
                                  (const int32_t *)pt.p, &qs);
    unpin(e, &ty); unpin(e, &io); unpin(e, &ic); unpin(e, &ho); unpin(e, &po); unpin(e, &pt);
    if (ok && rc) throw_rc(e, rc);
    return ok && !rc ? (jlong)(intptr_t)qs : 0;
}

JNIEXPORT jlong JFN(patternBatchSet)(JNIEnv *e, jclass k, jlong g, jlong set) {
    hgx_query_result *q = NULL;
    int rc = hgx_pattern_batch_set((hgx_graph *)(intptr_t)g, (const hgx_query_set *)(intptr_t)set, &q);
    if (rc) { throw_rc(e, rc); return 0; }
    return (jlong)(intptr_t)q;
}

JNIEXPORT void JFN(querySetFree)(JNIEnv *e, jclass k, jlong set) { hgx_query_set_free((hgx_query_set *)(intptr_t)set); }

/* The set's results into caller arrays: offsets (n + 1 entries) always, ids when they fit; returns the
 * number of hits (a larger ids array and a second call when it exceeds ids.length). */
JNIEXPORT jlong JFN(patternBatchSetInto)(JNIEnv *e, jclass k, jlong g, jlong set, jlongArray offsets, jintArray ids) {
    if (!check_not_null(e, offsets, "offsets")) return 0;
    int32_t nq = 0;   /* the engine writes nq + 1 offsets: a shorter array is refused before the call */
    int rc = hgx_query_set_info((const hgx_query_set *)(intptr_t)set, &nq);
    if (rc) { throw_rc(e, rc); return 0; }
    pin_t off = pin_long(e, offsets), id = pin_int(e, ids);
    int64_t n_ids = 0;
    int ok = !pin_failed(&off) && !pin_failed(&id) && check_len(e, &off, (int64_t)nq + 1, "offsets");
    if (ok)
        rc = hgx_pattern_batch_set_into((hgx_graph *)(intptr_t)g, (const hgx_query_set *)(intptr_t)set,
                                        (int64_t *)off.p, (int32_t *)id.p, (int64_t)id.n, &n_ids, NULL);
    unpin_out(e, &off); unpin_out(e, &id);
    if (ok && rc) throw_rc(e, rc);
    return ok && !rc ? (jlong)n_ids : 0;
}

JNIEXPORT jlong JFN(patternBatchExt)(JNIEnv *e, jclass k, jlong g, jlongArray typeOff, jintArray types,
                                     jlongArray incOff, jintArray inc, jlongArray posOff, jintArray pos,
                                     jlongArray psetOff, jlongArray patOff, jintArray pat, jintArray arity) {
    pin_t to = pin_long(e, typeOff), ty = pin_int(e, types), io = pin_long(e, incOff), ic = pin_int(e, inc),
          po = pin_long(e, posOff), ps = pin_int(e, pos), so = pin_long(e, psetOff), pa = pin_long(e, patOff),
          pt = pin_int(e, pat), ar = pin_int(e, arity);
    const jsize n = ar.n;
    hgx_query_result *q = NULL;
    int rc = HGX_OK;
    /* psetOff indexes the orderedLink patterns, each of which is a slice of pat through patOff
     * (psetOff[n] + 1 entries); a positioned record is 4 ints of pos */
    int ok = !pin_failed(&ar) && !pin_failed(&ty) && !pin_failed(&ic) && !pin_failed(&ps) && !pin_failed(&pt) &&
             check_offsets(e, &to, (int64_t)n + 1, ty.n, 1, "typeOff") &&
             check_offsets(e, &io, (int64_t)n + 1, ic.n, 1, "incOff") &&
             check_offsets(e, &po, (int64_t)n + 1, ps.n, 4, "posOff") &&
             check_offsets(e, &so, (int64_t)n + 1, pa.n > 0 ? (int64_t)pa.n - 1 : 0, 1, "psetOff");
    if (ok) {
        const int64_t nsets = so.n ? ((const int64_t *)so.p)[n] : 0;
        ok = (nsets == 0 && pa.n == 0) || check_offsets(e, &pa, nsets + 1, pt.n, 1, "patOff");
    }
    if (ok)
        rc = hgx_pattern_batch_ext((hgx_graph *)(intptr_t)g, n, (const int64_t *)to.p, (const int32_t *)ty.p,
                                   (const int64_t *)io.p, (const int32_t *)ic.p, (const int64_t *)po.p,
                                   (const int32_t *)ps.p, (const int64_t *)so.p, (const int64_t *)pa.p,
                                   (const int32_t *)pt.p, (const int32_t *)ar.p, &q);
    unpin(e, &to); unpin(e, &ty); unpin(e, &io); unpin(e, &ic); unpin(e, &po);
    unpin(e, &ps); unpin(e, &so); unpin(e, &pa); unpin(e, &pt); unpin(e, &ar);
    if (ok && rc) throw_rc(e, rc);
    return ok && !rc ? (jlong)(intptr_t)q : 0;
}

JNIEXPORT jlongArray JFN(queryOffsets)(JNIEnv *e, jclass k, jlong qr) {
    const hgx_query_result *q = (const hgx_query_result *)(intptr_t)qr;
    int64_t count = 0;
    int rc = hgx_query_result_count(q, &count);
    if (rc) { throw_rc(e, rc); return NULL; }
    if (!fits_jarray(e, count + 1, "queryOffsets")) return NULL;
    int64_t *off = (int64_t *)malloc(sizeof(int64_t) * (size_t)(count + 1));
    rc = off ? hgx_query_result_offsets(q, off) : HGX_E_NOMEM;
    jlongArray out = rc ? NULL : new_longs(e, off, count + 1);
    free(off);
    if (rc) throw_rc(e, rc);
    return out;
}

JNIEXPORT jintArray JFN(queryIds)(JNIEnv *e, jclass k, jlong qr) {
    const hgx_query_result *q = (const hgx_query_result *)(intptr_t)qr;
    int64_t count = 0, total = 0;
    int rc = hgx_query_result_count(q, &count);
    if (!rc) {
        int64_t *off = (int64_t *)malloc(sizeof(int64_t) * (size_t)(count + 1));
        rc = off ? hgx_query_result_offsets(q, off) : HGX_E_NOMEM;
        if (!rc) total = off[count];
        free(off);
    }
    if (rc) { throw_rc(e, rc); return NULL; }
    if (!fits_jarray(e, total, "queryIds")) return NULL;
    int32_t *ids = (int32_t *)malloc(sizeof(int32_t) * (size_t)(total > 0 ? total : 1));
    rc = ids ? hgx_query_result_ids(q, ids) : HGX_E_NOMEM;
    jintArray out = rc ? NULL : new_ints(e, ids, total);
    free(ids);
    if (rc) throw_rc(e, rc);
    return out;
}

JNIEXPORT void JFN(queryFree)(JNIEnv *e, jclass k, jlong q) { hgx_query_result_free((hgx_query_result *)(intptr_t)q); }

JNIEXPORT jlongArray JFN(queryCoalesceStats)(JNIEnv *e, jclass k, jlong g) {
    int64_t v[2] = {0, 0};
    int rc = hgx_query_coalesce_stats((hgx_graph *)(intptr_t)g, &v[0], &v[1]);
    if (rc) { throw_rc(e, rc); return NULL; }
    return new_longs(e, v, 2);
}

/* ---- partitioned snapshot -------------------------------------------------------------------- */

JNIEXPORT jintArray JFN(partitionPlan)(JNIEnv *e, jclass k, jlong numAtoms, jintArray linkAtom, jlongArray tgtOff,
                                       jintArray tgtIdx, jintArray linkType, jint nParts) {
    pin_t la = pin_int(e, linkAtom), off = pin_long(e, tgtOff), tg = pin_int(e, tgtIdx), ty = pin_int(e, linkType);
    int ok = check_rows(e, &la, &off, &tg, &ty), rc = HGX_OK;
    int32_t *plan = NULL;
    jintArray out = NULL;
    if (ok) {
        plan = (int32_t *)malloc(sizeof(int32_t) * (size_t)(la.n > 0 ? la.n : 1));
        hgx_graph_desc d = desc_of(numAtoms, &la, &off, &tg, &ty);
        rc = !plan ? HGX_E_NOMEM : hgx_partition_plan(&d, nParts, plan);
        if (!rc) out = new_ints(e, plan, la.n);
    }
    unpin(e, &la); unpin(e, &off); unpin(e, &tg); unpin(e, &ty);
    free(plan);
    if (ok && rc) throw_rc(e, rc);
    return out;
}

JNIEXPORT jlong JFN(shardBuild)(JNIEnv *e, jclass k, jlong numAtoms, jintArray linkAtom, jlongArray tgtOff,
                                jintArray tgtIdx, jintArray linkType, jint nParts, jint part, jintArray plan) {
    pin_t la = pin_int(e, linkAtom), off = pin_long(e, tgtOff), tg = pin_int(e, tgtIdx), ty = pin_int(e, linkType),
          pl = pin_int(e, plan);
    hgx_shard *s = NULL;
    int ok = check_rows(e, &la, &off, &tg, &ty) && check_len(e, &pl, la.n, "plan"), rc = HGX_OK;
    if (ok) {
        hgx_graph_desc d = desc_of(numAtoms, &la, &off, &tg, &ty);
        rc = hgx_shard_build(&d, nParts, part, (const int32_t *)pl.p, &s);
    }
    unpin(e, &la); unpin(e, &off); unpin(e, &tg); unpin(e, &ty); unpin(e, &pl);
    if (ok && rc) throw_rc(e, rc);
    return ok && !rc ? (jlong)(intptr_t)s : 0;
}

JNIEXPORT void JFN(shardFree)(JNIEnv *e, jclass k, jlong s) { hgx_shard_free((hgx_shard *)(intptr_t)s); }

JNIEXPORT jlong JFN(shardGraphCreate)(JNIEnv *e, jclass k, jlong s, jint device) {
    hgx_graph *g = NULL;
    int rc = hgx_shard_graph_create((const hgx_shard *)(intptr_t)s, device, &g);
    if (rc) { throw_rc(e, rc); return 0; }
    return (jlong)(intptr_t)g;
}

JNIEXPORT jbyteArray JFN(rcclUniqueId)(JNIEnv *e, jclass k) {
    uint8_t id[128];
    int rc = hgx_comm_rccl_unique_id(id);
    if (rc) { throw_rc(e, rc); return NULL; }
    jbyteArray out = (*e)->NewByteArray(e, 128);
    if (out) (*e)->SetByteArrayRegion(e, out, 0, 128, (const jbyte *)id);
    return out;
}

JNIEXPORT jlong JFN(rcclCreate)(JNIEnv *e, jclass k, jbyteArray id, jint world, jint rank, jint device) {
    if (!id || (*e)->GetArrayLength(e, id) != 128) { throw_msg(e, "RCCL unique id must be 128 bytes"); return 0; }
    uint8_t buf[128];
    (*e)->GetByteArrayRegion(e, id, 0, 128, (jbyte *)buf);
    hgx_comm *c = NULL;
    int rc = hgx_comm_rccl_create(buf, world, rank, device, &c);
    if (rc) { throw_rc(e, rc); return 0; }
    return (jlong)(intptr_t)c;
}

JNIEXPORT void JFN(commDestroy)(JNIEnv *e, jclass k, jlong c) { hgx_comm_destroy((hgx_comm *)(intptr_t)c); }

JNIEXPORT jlong JFN(pbfsBatch)(JNIEnv *e, jclass k, jlong shard, jlong comm, jintArray seeds, jint maxDepth,
                               jint linkType, jboolean p, jboolean s, jboolean r, jboolean src) {
    pin_t sd = pin_int(e, seeds);
    if (pin_failed(&sd)) return 0;
    hgx_algen_opts o = opts_of(linkType, p, s, r, src);
    hgx_bfs_result *res = NULL;
    int rc = hgx_pbfs_batch((hgx_graph *)(intptr_t)shard, (hgx_comm *)(intptr_t)comm, (const int32_t *)sd.p, sd.n,
                            maxDepth, &o, &res);
    unpin(e, &sd);
    if (rc) { throw_rc(e, rc); return 0; }
    return (jlong)(intptr_t)res;
}

JNIEXPORT jlongArray JFN(shardInfo)(JNIEnv *e, jclass k, jlong sh) {
    int64_t v[4];
    int rc = hgx_shard_info((const hgx_shard *)(intptr_t)sh, &v[0], &v[1], &v[2], &v[3]);
    if (rc) { throw_rc(e, rc); return NULL; }
    return new_longs(e, v, 4);
}

JNIEXPORT jintArray JFN(shardLocalAtoms)(JNIEnv *e, jclass k, jlong sh) {
    const hgx_shard *s = (const hgx_shard *)(intptr_t)sh;
    int64_t nl = 0;
    int rc = hgx_shard_info(s, &nl, NULL, NULL, NULL);
    if (rc) { throw_rc(e, rc); return NULL; }
    if (!fits_jarray(e, nl, "shardLocalAtoms")) return NULL;
    int32_t *l2g = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nl > 0 ? nl : 1));
    rc = l2g ? hgx_shard_export(s, l2g, NULL, NULL, NULL, NULL, NULL) : HGX_E_NOMEM;
    jintArray out = rc ? NULL : new_ints(e, l2g, nl);
    free(l2g);
    if (rc) throw_rc(e, rc);
    return out;
}

JNIEXPORT jintArray JFN(shardOwners)(JNIEnv *e, jclass k, jlong sh) {
    const hgx_shard *s = (const hgx_shard *)(intptr_t)sh;
    int64_t nl = 0;
    int rc = hgx_shard_info(s, &nl, NULL, NULL, NULL);
    if (rc) { throw_rc(e, rc); return NULL; }
    if (!fits_jarray(e, nl, "shardOwners")) return NULL;
    int32_t *xo = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nl > 0 ? nl : 1));
    rc = xo ? hgx_shard_exchange_tables(s, xo, NULL, NULL, NULL, NULL, NULL) : HGX_E_NOMEM;
    jintArray out = rc ? NULL : new_ints(e, xo, nl);
    free(xo);
    if (rc) throw_rc(e, rc);
    return out;
}

JNIEXPORT jlongArray JFN(pbfsBatchGroup)(JNIEnv *e, jclass k, jlongArray shards, jintArray seeds, jint maxDepth,
                                         jint linkType, jboolean p, jboolean s, jboolean r, jboolean src) {
    pin_t sh = pin_long(e, shards), sd = pin_int(e, seeds);
    hgx_algen_opts o = opts_of(linkType, p, s, r, src);
    const jsize np = sh.n;
    int ok = !pin_failed(&sh) && !pin_failed(&sd) && check_not_null(e, sh.a, "shards");
    hgx_graph **gs = NULL;
    hgx_bfs_result **outs = NULL;
    int rc = HGX_OK;
    jlongArray out = NULL;
    if (ok) {
        gs = (hgx_graph **)malloc(sizeof(hgx_graph *) * (size_t)(np > 0 ? np : 1));
        outs = (hgx_bfs_result **)calloc((size_t)(np > 0 ? np : 1), sizeof(hgx_bfs_result *));
        rc = (!gs || !outs) ? HGX_E_NOMEM : HGX_OK;
        for (jsize i = 0; !rc && i < np; i++) gs[i] = (hgx_graph *)(intptr_t)((const jlong *)sh.p)[i];
        if (!rc) rc = hgx_pbfs_batch_group(gs, np, (const int32_t *)sd.p, sd.n, maxDepth, &o, outs);
        if (!rc) {
            int64_t *h = (int64_t *)malloc(sizeof(int64_t) * (size_t)(np > 0 ? np : 1));
            if (h) {
                for (jsize i = 0; i < np; i++) h[i] = (int64_t)(intptr_t)outs[i];
                out = new_longs(e, h, np);
                free(h);
            }
            if (!out) {   /* the results cannot reach Java: free them (OutOfMemoryError pending or NOMEM) */
                for (jsize i = 0; i < np; i++) hgx_bfs_result_free(outs[i]);
                if (!h) rc = HGX_E_NOMEM;
            }
        }
    }
    unpin(e, &sh);
    unpin(e, &sd);
    free(gs);
    free(outs);
    if (ok && rc) throw_rc(e, rc);
    return out;
}

static jarray new_doubles(JNIEnv *e, const double *v, jsize n) {
    jarray a = (*e)->NewDoubleArray(e, n);
    if (a && n) (*e)->SetDoubleArrayRegion(e, a, 0, n, v);
    return a;
}

JNIEXPORT void JFN(setTiming)(JNIEnv *e, jclass k, jlong g, jboolean on) {
    int rc = hgx_set_timing((hgx_graph *)(intptr_t)g, on ? 1 : 0);
    if (rc) throw_rc(e, rc);
}

JNIEXPORT jarray JFN(bfsStats)(JNIEnv *e, jclass k, jlong r, jboolean accounting) {
    hgx_bfs_stats st;
    int rc = hgx_bfs_result_stats((hgx_bfs_result *)(intptr_t)r, accounting ? 1 : 0, &st);
    if (rc) { throw_rc(e, rc); return NULL; }
    double v[5] = {st.ms_total, st.traversed_edges, st.bytes_min, st.ms_exchange, st.bytes_exchanged};
    return new_doubles(e, v, 5);
}

JNIEXPORT jarray JFN(seqStats)(JNIEnv *e, jclass k, jlong sq) {
    double v[2] = {0, 0};
    int rc = hgx_seq_result_stats((const hgx_seq_result *)(intptr_t)sq, &v[0], &v[1]);
    if (rc) { throw_rc(e, rc); return NULL; }
    return new_doubles(e, v, 2);
}

JNIEXPORT jlongArray JFN(seqEngineStats)(JNIEnv *e, jclass k, jlong sq) {
    int32_t nb = 0, nl = 0;
    int64_t pl = 0;
    int rc = hgx_seq_result_engine_stats((const hgx_seq_result *)(intptr_t)sq, &nb, &nl, NULL, NULL);
    int32_t nc = 0;
    if (!rc) rc = hgx_seq_result_level_stats((const hgx_seq_result *)(intptr_t)sq, NULL, NULL, &pl);
    if (!rc) rc = hgx_seq_result_grid_stats((const hgx_seq_result *)(intptr_t)sq, &nc, NULL, NULL);
    if (rc) { throw_rc(e, rc); return NULL; }
    int64_t v[4] = {nb, nl, pl, nc};
    return new_longs(e, v, 4);
}

JNIEXPORT jarray JFN(queryMs)(JNIEnv *e, jclass k, jlong q) {
    double v[3] = {0, 0, 0};
    int rc = hgx_query_result_ms((const hgx_query_result *)(intptr_t)q, &v[0], &v[1], &v[2]);
    if (rc) { throw_rc(e, rc); return NULL; }
    return new_doubles(e, v, 3);
}

/* which: 0 link_atom, 1 tgt_idx */
static jintArray export_ints(JNIEnv *e, jlong gh, int which) {
    hgx_graph *g = (hgx_graph *)(intptr_t)gh;
    int64_t A = 0, M = 0, I = 0;
    int rc = hgx_graph_info(g, &A, &M, &I);
    if (rc) { throw_rc(e, rc); return NULL; }
    int64_t *off = (int64_t *)malloc(sizeof(int64_t) * (size_t)(M + 1));
    rc = off ? hgx_graph_export(g, NULL, off, NULL, NULL) : HGX_E_NOMEM;
    int64_t n = rc ? 0 : (which == 0 ? M : off[M]);
    free(off);
    if (rc) { throw_rc(e, rc); return NULL; }
    if (!fits_jarray(e, n, which == 0 ? "graphExportLinks" : "graphExportTargets")) return NULL;
    int32_t *buf = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    rc = buf ? hgx_graph_export(g, which == 0 ? buf : NULL, NULL, which == 1 ? buf : NULL, NULL) : HGX_E_NOMEM;
    jintArray out = rc ? NULL : new_ints(e, buf, n);
    free(buf);
    if (rc) throw_rc(e, rc);
    return out;
}

JNIEXPORT jintArray JFN(graphExportLinks)(JNIEnv *e, jclass k, jlong g) { return export_ints(e, g, 0); }
JNIEXPORT jintArray JFN(graphExportTargets)(JNIEnv *e, jclass k, jlong g) { return export_ints(e, g, 1); }

JNIEXPORT jlongArray JFN(graphExportOffsets)(JNIEnv *e, jclass k, jlong gh) {
    hgx_graph *g = (hgx_graph *)(intptr_t)gh;
    int64_t A = 0, M = 0, I = 0;
    int rc = hgx_graph_info(g, &A, &M, &I);
    if (rc) { throw_rc(e, rc); return NULL; }
    if (!fits_jarray(e, M + 1, "graphExportOffsets")) return NULL;
    int64_t *off = (int64_t *)malloc(sizeof(int64_t) * (size_t)(M + 1));
    rc = off ? hgx_graph_export(g, NULL, off, NULL, NULL) : HGX_E_NOMEM;
    jlongArray out = rc ? NULL : new_longs(e, off, M + 1);
    free(off);
    if (rc) throw_rc(e, rc);
    return out;
}

JNIEXPORT jlong JFN(patternBatchStructs)(JNIEnv *e, jclass k, jlong g, jintArray type, jlongArray incOff,
                                         jintArray inc, jintArray hasOrdered, jlongArray patOff, jintArray pat) {
    pin_t ty = pin_int(e, type), io = pin_long(e, incOff), ic = pin_int(e, inc), ho = pin_int(e, hasOrdered),
          po = pin_long(e, patOff), pt = pin_int(e, pat);
    const jsize n = ty.n;
    hgx_query_result *q = NULL;
    int ok = check_packed(e, &ty, &io, &ic, &ho, &po, &pt), rc = HGX_OK;
    hgx_and_query *qs = NULL;
    if (ok) {   /* the offsets are checked: every slice below lies inside inc / pat */
        qs = (hgx_and_query *)malloc(sizeof(hgx_and_query) * (size_t)(n > 0 ? n : 1));
        rc = qs ? HGX_OK : HGX_E_NOMEM;
        for (jsize i = 0; !rc && i < n; i++) {
            const int64_t *iof = (const int64_t *)io.p, *pof = (const int64_t *)po.p;
            qs[i].type = ((const int32_t *)ty.p)[i];
            qs[i].n_incident = (int32_t)(iof[i + 1] - iof[i]);
            qs[i].incident = (const int32_t *)ic.p + iof[i];
            qs[i].has_ordered = ((const int32_t *)ho.p)[i];
            qs[i].n_pattern = (int32_t)(pof[i + 1] - pof[i]);
            qs[i].pattern = (const int32_t *)pt.p + pof[i];
        }
        if (!rc) rc = hgx_pattern_batch((hgx_graph *)(intptr_t)g, qs, n, &q);
    }
    unpin(e, &ty); unpin(e, &io); unpin(e, &ic); unpin(e, &ho); unpin(e, &po); unpin(e, &pt);
    free(qs);
    if (ok && rc) throw_rc(e, rc);
    return ok && !rc ? (jlong)(intptr_t)q : 0;
}

JNIEXPORT jint JFN(deviceCount)(JNIEnv *e, jclass k) {
    int32_t n = 0;
    int rc = hgx_device_count(&n);
    if (rc) throw_rc(e, rc);
    return n;
}

JNIEXPORT void JFN(deviceSynchronize)(JNIEnv *e, jclass k, jint device) {
    int rc = hgx_device_synchronize(device);
    if (rc) throw_rc(e, rc);
}

JNIEXPORT jstring JFN(lastError)(JNIEnv *e, jclass k) { return (*e)->NewStringUTF(e, hgx_last_error()); }
JNIEXPORT jstring JFN(version)(JNIEnv *e, jclass k) { return (*e)->NewStringUTF(e, hgx_version()); }
