/*
 * hgx_jni.c -- JNI shim between org.hypergraphdb.gpu.Hgx (java/org/hypergraphdb/gpu/Hgx.java) and
 * the C ABI of libhgx.so (include/hgx.h).  Arrays in, handles (jlong) out; a nonzero status becomes
 * an exception: HGX_E_UNSUPPORTED -> java.lang.UnsupportedOperationException (the Java caller keeps
 * the reference class), anything else -> org.hypergraphdb.HGException with hgx_last_error().
 * Primitive arrays are pinned with Get<T>ArrayElements and released with JNI_ABORT (the ABI
 * deep-copies every input); no pointer into the JVM heap outlives a call, and nothing calls back
 * into the JVM (ownership).
 *
 * Build (a host with a JDK):
 *   gcc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *       java/jni/hgx_jni.c -Lhypergraphdb_amd -lhgx -Wl,-rpath,'$ORIGIN' -o libhgx_jni.so
 *
 * UNVERIFIED on a JVM: no JDK exists in this build image.  The C is
 * type-checked here against a minimal JNI declaration set (tests/test_abi.py::test_jni_shim_compiles),
 * never linked against a JVM or run.
 */
#include <jni.h>
#include <stdlib.h>
#include <string.h>

#include "hgx.h"

#define JFN(name) JNICALL Java_org_hypergraphdb_gpu_Hgx_##name

static void throw_rc(JNIEnv *e, int rc) {
    const char *cls = rc == HGX_E_UNSUPPORTED ? "java/lang/UnsupportedOperationException"
                    : rc == HGX_E_NOMEM       ? "java/lang/OutOfMemoryError"
                                              : "org/hypergraphdb/HGException";
    jclass c = (*e)->FindClass(e, cls);
    if (c) (*e)->ThrowNew(e, c, hgx_last_error());
}

static void throw_msg(JNIEnv *e, const char *msg) {
    jclass c = (*e)->FindClass(e, "java/lang/IllegalArgumentException");
    if (c) (*e)->ThrowNew(e, c, msg);
}

/* Pinned views of Java arrays (NULL array -> NULL pointer, length 0). */
typedef struct { jarray a; void *p; jsize n; int kind; } pin_t;   /* kind: 0 int, 1 long, 2 byte */

static pin_t pin_int(JNIEnv *e, jintArray a) {
    pin_t r = {a, NULL, 0, 0};
    if (a) { r.n = (*e)->GetArrayLength(e, a); r.p = (*e)->GetIntArrayElements(e, a, NULL); }
    return r;
}
static pin_t pin_long(JNIEnv *e, jlongArray a) {
    pin_t r = {a, NULL, 0, 1};
    if (a) { r.n = (*e)->GetArrayLength(e, a); r.p = (*e)->GetLongArrayElements(e, a, NULL); }
    return r;
}
static pin_t pin_byte(JNIEnv *e, jbyteArray a) {
    pin_t r = {a, NULL, 0, 2};
    if (a) { r.n = (*e)->GetArrayLength(e, a); r.p = (*e)->GetByteArrayElements(e, a, NULL); }
    return r;
}
static void unpin(JNIEnv *e, pin_t *x) {
    if (!x->a || !x->p) return;
    if (x->kind == 0) (*e)->ReleaseIntArrayElements(e, (jintArray)x->a, (jint *)x->p, JNI_ABORT);
    else if (x->kind == 1) (*e)->ReleaseLongArrayElements(e, (jlongArray)x->a, (jlong *)x->p, JNI_ABORT);
    else (*e)->ReleaseByteArrayElements(e, (jbyteArray)x->a, (jbyte *)x->p, JNI_ABORT);
    x->p = NULL;
}

static jintArray new_ints(JNIEnv *e, const int32_t *v, jsize n) {
    jintArray a = (*e)->NewIntArray(e, n);
    if (a && n) (*e)->SetIntArrayRegion(e, a, 0, n, (const jint *)v);
    return a;
}
static jlongArray new_longs(JNIEnv *e, const int64_t *v, jsize n) {
    jlongArray a = (*e)->NewLongArray(e, n);
    if (a && n) (*e)->SetLongArrayRegion(e, a, 0, n, (const jlong *)v);
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

/* ---- snapshot ------------------------------------------------------------------------------ */

JNIEXPORT jlong JFN(graphCreate)(JNIEnv *e, jclass k, jlong numAtoms, jintArray linkAtom, jlongArray tgtOff,
                                 jintArray tgtIdx, jintArray linkType, jint device) {
    pin_t la = pin_int(e, linkAtom), off = pin_long(e, tgtOff), tg = pin_int(e, tgtIdx), ty = pin_int(e, linkType);
    hgx_graph *g = NULL;
    int rc;
    if (off.n != la.n + 1 || (ty.a && ty.n != la.n)) rc = HGX_E_INVALID;
    else {
        hgx_graph_desc d = desc_of(numAtoms, &la, &off, &tg, &ty);
        rc = hgx_graph_create(&d, device, &g);
    }
    unpin(e, &la); unpin(e, &off); unpin(e, &tg); unpin(e, &ty);
    if (rc) { throw_rc(e, rc); return 0; }
    return (jlong)(intptr_t)g;
}

JNIEXPORT jlong JFN(graphOpen)(JNIEnv *e, jclass k, jstring path, jint device) {
    const char *p = (*e)->GetStringUTFChars(e, path, NULL);
    hgx_graph *g = NULL;
    int rc = hgx_graph_open(p, device, &g);
    (*e)->ReleaseStringUTFChars(e, path, p);
    if (rc) { throw_rc(e, rc); return 0; }
    return (jlong)(intptr_t)g;
}

JNIEXPORT void JFN(graphDestroy)(JNIEnv *e, jclass k, jlong g) { hgx_graph_destroy((hgx_graph *)(intptr_t)g); }

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
    int rc = (la.n && off.n != la.n + 1) ? HGX_E_INVALID
           : hgx_graph_update((hgx_graph *)(intptr_t)g, numAtoms, la.n, (const int32_t *)la.p, (const int64_t *)off.p,
                              (const int32_t *)tg.p, (const int32_t *)ty.p, rm.n, (const int32_t *)rm.p);
    unpin(e, &la); unpin(e, &off); unpin(e, &tg); unpin(e, &ty); unpin(e, &rm);
    if (rc) throw_rc(e, rc);
}

JNIEXPORT jintArray JFN(incidence)(JNIEnv *e, jclass k, jlong g, jint atom) {
    int64_t n = 0;
    int rc = hgx_graph_incidence((hgx_graph *)(intptr_t)g, atom, NULL, 0, &n);
    if (rc) { throw_rc(e, rc); return NULL; }
    int32_t *buf = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    if (!buf) { throw_rc(e, HGX_E_NOMEM); return NULL; }
    rc = hgx_graph_incidence((hgx_graph *)(intptr_t)g, atom, buf, n, &n);
    jintArray out = rc ? NULL : new_ints(e, buf, (jsize)n);
    free(buf);
    if (rc) throw_rc(e, rc);
    return out;
}

JNIEXPORT jlongArray JFN(degree)(JNIEnv *e, jclass k, jlong g, jintArray atoms) {
    pin_t a = pin_int(e, atoms);
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
    pin_t la = pin_int(e, linkAtom), off = pin_long(e, tgtOff), tg = pin_int(e, tgtIdx), ty = pin_int(e, linkType),
          hb = pin_byte(e, handles);
    const char *p = (*e)->GetStringUTFChars(e, path, NULL);
    hgx_graph_desc d = desc_of(numAtoms, &la, &off, &tg, &ty);
    int rc = (off.n != la.n + 1) ? HGX_E_INVALID
           : hgx_snapshot_write(p, &d, (const uint8_t *)hb.p, hb.p ? handleBytes : 0);
    (*e)->ReleaseStringUTFChars(e, path, p);
    unpin(e, &la); unpin(e, &off); unpin(e, &tg); unpin(e, &ty); unpin(e, &hb);
    if (rc) throw_rc(e, rc);
}

JNIEXPORT jlongArray JFN(snapshotInfo)(JNIEnv *e, jclass k, jstring path) {
    const char *p = (*e)->GetStringUTFChars(e, path, NULL);
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
    const char *p = (*e)->GetStringUTFChars(e, path, NULL);
    int64_t A = 0;
    int32_t hb = 0;
    int rc = hgx_snapshot_info(p, &A, NULL, NULL, &hb, NULL);
    jbyteArray out = NULL;
    if (!rc && hb > 0) {
        uint8_t *buf = (uint8_t *)malloc((size_t)A * (size_t)hb);
        rc = buf ? hgx_snapshot_read(p, NULL, NULL, NULL, NULL, buf) : HGX_E_NOMEM;
        if (!rc) {
            out = (*e)->NewByteArray(e, (jsize)(A * hb));
            if (out) (*e)->SetByteArrayRegion(e, out, 0, (jsize)(A * hb), (const jbyte *)buf);
        }
        free(buf);
    }
    (*e)->ReleaseStringUTFChars(e, path, p);
    if (rc) throw_rc(e, rc);
    return out;
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
    int64_t *c = (int64_t *)malloc(sizeof(int64_t) * ((size_t)ns * nl + 1));
    rc = c ? hgx_bfs_result_counts((hgx_bfs_result *)(intptr_t)r, c) : HGX_E_NOMEM;
    jlongArray out = rc ? NULL : new_longs(e, c, ns * nl);
    free(c);
    if (rc) throw_rc(e, rc);
    return out;
}

JNIEXPORT jintArray JFN(bfsVisited)(JNIEnv *e, jclass k, jlong r, jint seedIndex, jint depth) {
    int64_t n = 0;
    hgx_bfs_result *res = (hgx_bfs_result *)(intptr_t)r;
    int rc = hgx_bfs_result_visited(res, seedIndex, depth, NULL, 0, &n);
    if (rc) { throw_rc(e, rc); return NULL; }
    int32_t *buf = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    rc = buf ? hgx_bfs_result_visited(res, seedIndex, depth, buf, n, &n) : HGX_E_NOMEM;
    jintArray out = rc ? NULL : new_ints(e, buf, (jsize)n);
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
    jlongArray out = rc ? NULL : new_longs(e, off, ns + 1);
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
    int32_t *buf = (int32_t *)malloc(sizeof(int32_t) * (size_t)(np > 0 ? np : 1));
    if (!buf) { throw_rc(e, HGX_E_NOMEM); return NULL; }
    rc = hgx_seq_result_pairs(s, which == 0 ? buf : NULL, which == 1 ? buf : NULL, which == 2 ? buf : NULL);
    jintArray out = rc ? NULL : new_ints(e, buf, (jsize)np);
    free(buf);
    if (rc) throw_rc(e, rc);
    return out;
}

JNIEXPORT jintArray JFN(seqLinks)(JNIEnv *e, jclass k, jlong s) { return seq_column(e, s, 0); }
JNIEXPORT jintArray JFN(seqAtoms)(JNIEnv *e, jclass k, jlong s) { return seq_column(e, s, 1); }
JNIEXPORT jintArray JFN(seqDists)(JNIEnv *e, jclass k, jlong s) { return seq_column(e, s, 2); }
JNIEXPORT void JFN(seqFree)(JNIEnv *e, jclass k, jlong s) { hgx_seq_result_free((hgx_seq_result *)(intptr_t)s); }

/* ---- conjunctive pattern batches ------------------------------------------------------------- */

JNIEXPORT jlong JFN(patternBatch)(JNIEnv *e, jclass k, jlong g, jintArray type, jlongArray incOff, jintArray inc,
                                  jintArray hasOrdered, jlongArray patOff, jintArray pat) {
    pin_t ty = pin_int(e, type), io = pin_long(e, incOff), ic = pin_int(e, inc), ho = pin_int(e, hasOrdered),
          po = pin_long(e, patOff), pt = pin_int(e, pat);
    hgx_query_result *q = NULL;
    int rc = (io.n != ty.n + 1 || po.n != ty.n + 1 || ho.n != ty.n) ? HGX_E_INVALID
           : hgx_pattern_batch_packed((hgx_graph *)(intptr_t)g, ty.n, (const int32_t *)ty.p, (const int64_t *)io.p,
                                      (const int32_t *)ic.p, (const int32_t *)ho.p, (const int64_t *)po.p,
                                      (const int32_t *)pt.p, &q);
    unpin(e, &ty); unpin(e, &io); unpin(e, &ic); unpin(e, &ho); unpin(e, &po); unpin(e, &pt);
    if (rc) { throw_rc(e, rc); return 0; }
    return (jlong)(intptr_t)q;
}

JNIEXPORT jlong JFN(patternBatchExt)(JNIEnv *e, jclass k, jlong g, jlongArray typeOff, jintArray types,
                                     jlongArray incOff, jintArray inc, jlongArray posOff, jintArray pos,
                                     jlongArray psetOff, jlongArray patOff, jintArray pat, jintArray arity) {
    pin_t to = pin_long(e, typeOff), ty = pin_int(e, types), io = pin_long(e, incOff), ic = pin_int(e, inc),
          po = pin_long(e, posOff), ps = pin_int(e, pos), so = pin_long(e, psetOff), pa = pin_long(e, patOff),
          pt = pin_int(e, pat), ar = pin_int(e, arity);
    const jsize n = ar.n;
    hgx_query_result *q = NULL;
    int rc = (to.n != n + 1 || io.n != n + 1 || po.n != n + 1 || so.n != n + 1) ? HGX_E_INVALID
           : hgx_pattern_batch_ext((hgx_graph *)(intptr_t)g, n, (const int64_t *)to.p, (const int32_t *)ty.p,
                                   (const int64_t *)io.p, (const int32_t *)ic.p, (const int64_t *)po.p,
                                   (const int32_t *)ps.p, (const int64_t *)so.p, (const int64_t *)pa.p,
                                   (const int32_t *)pt.p, (const int32_t *)ar.p, &q);
    unpin(e, &to); unpin(e, &ty); unpin(e, &io); unpin(e, &ic); unpin(e, &po);
    unpin(e, &ps); unpin(e, &so); unpin(e, &pa); unpin(e, &pt); unpin(e, &ar);
    if (rc) { throw_rc(e, rc); return 0; }
    return (jlong)(intptr_t)q;
}

JNIEXPORT jlongArray JFN(queryOffsets)(JNIEnv *e, jclass k, jlong qr) {
    const hgx_query_result *q = (const hgx_query_result *)(intptr_t)qr;
    int64_t count = 0;
    int rc = hgx_query_result_count(q, &count);
    if (rc) { throw_rc(e, rc); return NULL; }
    int64_t *off = (int64_t *)malloc(sizeof(int64_t) * (size_t)(count + 1));
    rc = off ? hgx_query_result_offsets(q, off) : HGX_E_NOMEM;
    jlongArray out = rc ? NULL : new_longs(e, off, (jsize)(count + 1));
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
    int32_t *ids = (int32_t *)malloc(sizeof(int32_t) * (size_t)(total > 0 ? total : 1));
    rc = ids ? hgx_query_result_ids(q, ids) : HGX_E_NOMEM;
    jintArray out = rc ? NULL : new_ints(e, ids, (jsize)total);
    free(ids);
    if (rc) throw_rc(e, rc);
    return out;
}

JNIEXPORT void JFN(queryFree)(JNIEnv *e, jclass k, jlong q) { hgx_query_result_free((hgx_query_result *)(intptr_t)q); }

/* ---- partitioned snapshot -------------------------------------------------------------------- */

JNIEXPORT jintArray JFN(partitionPlan)(JNIEnv *e, jclass k, jlong numAtoms, jintArray linkAtom, jlongArray tgtOff,
                                       jintArray tgtIdx, jintArray linkType, jint nParts) {
    pin_t la = pin_int(e, linkAtom), off = pin_long(e, tgtOff), tg = pin_int(e, tgtIdx), ty = pin_int(e, linkType);
    int32_t *plan = (int32_t *)malloc(sizeof(int32_t) * (size_t)(la.n > 0 ? la.n : 1));
    hgx_graph_desc d = desc_of(numAtoms, &la, &off, &tg, &ty);
    int rc = !plan ? HGX_E_NOMEM : (off.n != la.n + 1) ? HGX_E_INVALID : hgx_partition_plan(&d, nParts, plan);
    jintArray out = rc ? NULL : new_ints(e, plan, la.n);
    unpin(e, &la); unpin(e, &off); unpin(e, &tg); unpin(e, &ty);
    free(plan);
    if (rc) throw_rc(e, rc);
    return out;
}

JNIEXPORT jlong JFN(shardBuild)(JNIEnv *e, jclass k, jlong numAtoms, jintArray linkAtom, jlongArray tgtOff,
                                jintArray tgtIdx, jintArray linkType, jint nParts, jint part, jintArray plan) {
    pin_t la = pin_int(e, linkAtom), off = pin_long(e, tgtOff), tg = pin_int(e, tgtIdx), ty = pin_int(e, linkType),
          pl = pin_int(e, plan);
    hgx_graph_desc d = desc_of(numAtoms, &la, &off, &tg, &ty);
    hgx_shard *s = NULL;
    int rc = (off.n != la.n + 1 || pl.n != la.n) ? HGX_E_INVALID
           : hgx_shard_build(&d, nParts, part, (const int32_t *)pl.p, &s);
    unpin(e, &la); unpin(e, &off); unpin(e, &tg); unpin(e, &ty); unpin(e, &pl);
    if (rc) { throw_rc(e, rc); return 0; }
    return (jlong)(intptr_t)s;
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
    int32_t *l2g = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nl > 0 ? nl : 1));
    rc = l2g ? hgx_shard_export(s, l2g, NULL, NULL, NULL, NULL, NULL) : HGX_E_NOMEM;
    jintArray out = rc ? NULL : new_ints(e, l2g, (jsize)nl);
    free(l2g);
    if (rc) throw_rc(e, rc);
    return out;
}

JNIEXPORT jintArray JFN(shardOwners)(JNIEnv *e, jclass k, jlong sh) {
    const hgx_shard *s = (const hgx_shard *)(intptr_t)sh;
    int64_t nl = 0;
    int rc = hgx_shard_info(s, &nl, NULL, NULL, NULL);
    if (rc) { throw_rc(e, rc); return NULL; }
    int32_t *xo = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nl > 0 ? nl : 1));
    rc = xo ? hgx_shard_exchange_tables(s, xo, NULL, NULL, NULL, NULL, NULL) : HGX_E_NOMEM;
    jintArray out = rc ? NULL : new_ints(e, xo, (jsize)nl);
    free(xo);
    if (rc) throw_rc(e, rc);
    return out;
}

JNIEXPORT jlongArray JFN(pbfsBatchGroup)(JNIEnv *e, jclass k, jlongArray shards, jintArray seeds, jint maxDepth,
                                         jint linkType, jboolean p, jboolean s, jboolean r, jboolean src) {
    pin_t sh = pin_long(e, shards), sd = pin_int(e, seeds);
    hgx_algen_opts o = opts_of(linkType, p, s, r, src);
    const jsize np = sh.n;
    hgx_graph **gs = (hgx_graph **)malloc(sizeof(hgx_graph *) * (size_t)(np > 0 ? np : 1));
    hgx_bfs_result **outs = (hgx_bfs_result **)calloc((size_t)(np > 0 ? np : 1), sizeof(hgx_bfs_result *));
    int rc = (!gs || !outs) ? HGX_E_NOMEM : HGX_OK;
    for (jsize i = 0; !rc && i < np; i++) gs[i] = (hgx_graph *)(intptr_t)((const jlong *)sh.p)[i];
    if (!rc) rc = hgx_pbfs_batch_group(gs, np, (const int32_t *)sd.p, sd.n, maxDepth, &o, outs);
    jlongArray out = NULL;
    if (!rc) {
        int64_t *h = (int64_t *)malloc(sizeof(int64_t) * (size_t)(np > 0 ? np : 1));
        if (h) {
            for (jsize i = 0; i < np; i++) h[i] = (int64_t)(intptr_t)outs[i];
            out = new_longs(e, h, np);
            free(h);
        } else {
            for (jsize i = 0; i < np; i++) hgx_bfs_result_free(outs[i]);
            rc = HGX_E_NOMEM;
        }
    }
    unpin(e, &sh);
    unpin(e, &sd);
    free(gs);
    free(outs);
    if (rc) throw_rc(e, rc);
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
    int32_t *buf = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    rc = buf ? hgx_graph_export(g, which == 0 ? buf : NULL, NULL, which == 1 ? buf : NULL, NULL) : HGX_E_NOMEM;
    jintArray out = rc ? NULL : new_ints(e, buf, (jsize)n);
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
    int64_t *off = (int64_t *)malloc(sizeof(int64_t) * (size_t)(M + 1));
    rc = off ? hgx_graph_export(g, NULL, off, NULL, NULL) : HGX_E_NOMEM;
    jlongArray out = rc ? NULL : new_longs(e, off, (jsize)(M + 1));
    free(off);
    if (rc) throw_rc(e, rc);
    return out;
}

JNIEXPORT jlong JFN(patternBatchStructs)(JNIEnv *e, jclass k, jlong g, jintArray type, jlongArray incOff,
                                         jintArray inc, jintArray hasOrdered, jlongArray patOff, jintArray pat) {
    pin_t ty = pin_int(e, type), io = pin_long(e, incOff), ic = pin_int(e, inc), ho = pin_int(e, hasOrdered),
          po = pin_long(e, patOff), pt = pin_int(e, pat);
    const jsize n = ty.n;
    hgx_and_query *qs = (hgx_and_query *)malloc(sizeof(hgx_and_query) * (size_t)(n > 0 ? n : 1));
    hgx_query_result *q = NULL;
    int rc = !qs ? HGX_E_NOMEM : (io.n != n + 1 || po.n != n + 1 || ho.n != n) ? HGX_E_INVALID : HGX_OK;
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
    unpin(e, &ty); unpin(e, &io); unpin(e, &ic); unpin(e, &ho); unpin(e, &po); unpin(e, &pt);
    free(qs);
    if (rc) { throw_rc(e, rc); return 0; }
    return (jlong)(intptr_t)q;
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
