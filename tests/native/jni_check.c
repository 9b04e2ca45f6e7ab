/*
 * jni_check.c -- TEST INFRASTRUCTURE: the JNI shim (java/jni/hgx_jni.c) under AddressSanitizer +
 * UBSan, driven through the test JNIEnv (tests/native/fake_jni.c) like a JVM would drive it.  Built by
 * `make -C hypergraphdb_amd/csrc sanitize` (build/san/jni_check, shim + env + engine host code all
 * sanitized) and run by tests/test_sanitize.py.  Only natives that need no GPU: version / errors, null
 * handles, the .hgcsr file natives, the partition planner and shard tables, and every argument check
 * the shim makes before the engine is called, each also with an OutOfMemoryError injected at every
 * pin.  After every call: no pin outstanding, no JNI-discipline violation recorded by the env.
 *
 *   build/san/jni_check <scratch dir>
 */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* the test env (tests/native/fake_jni.c) */
JNIEnv *fj_env_new(void);
void fj_env_free(JNIEnv *e);
jobject fj_new_array(JNIEnv *e, int kind, const void *data, int64_t n);
jobject fj_new_string(JNIEnv *e, const char *s);
int64_t fj_length(jobject o);
const void *fj_data(jobject o);
const char *fj_exception_class(JNIEnv *e);
const char *fj_exception_message(JNIEnv *e);
void fj_exception_clear(JNIEnv *e);
int64_t fj_outstanding_pins(JNIEnv *e);
int fj_violations(JNIEnv *e);
const char *fj_violation_text(JNIEnv *e);
void fj_inject_oom(JNIEnv *e, int64_t nth);

#define JN(name) Java_org_hypergraphdb_gpu_Hgx_##name
jstring JN(version)(JNIEnv *, jclass);
jstring JN(lastError)(JNIEnv *, jclass);
jlongArray JN(graphInfo)(JNIEnv *, jclass, jlong);
jintArray JN(bfsInfo)(JNIEnv *, jclass, jlong);
jlongArray JN(queryOffsets)(JNIEnv *, jclass, jlong);
jlongArray JN(shardInfo)(JNIEnv *, jclass, jlong);
jlongArray JN(seqOffsets)(JNIEnv *, jclass, jlong);
jlong JN(graphCreate)(JNIEnv *, jclass, jlong, jintArray, jlongArray, jintArray, jintArray, jint);
void JN(snapshotWrite)(JNIEnv *, jclass, jstring, jlong, jintArray, jlongArray, jintArray, jintArray, jbyteArray, jint);
jlongArray JN(snapshotInfo)(JNIEnv *, jclass, jstring);
jbyteArray JN(snapshotHandles)(JNIEnv *, jclass, jstring);
void JN(snapshotVerify)(JNIEnv *, jclass, jstring);
jbyteArray JN(snapshotHandlesRange)(JNIEnv *, jclass, jstring, jlong, jlong);
jlong JN(snapshotWriterBegin)(JNIEnv *, jclass, jstring, jlong, jintArray, jlongArray, jintArray, jintArray, jint);
void JN(snapshotWriterHandles)(JNIEnv *, jclass, jlong, jbyteArray, jint);
void JN(snapshotWriterEnd)(JNIEnv *, jclass, jlong);
void JN(snapshotWriterAbort)(JNIEnv *, jclass, jlong);
jintArray JN(partitionPlan)(JNIEnv *, jclass, jlong, jintArray, jlongArray, jintArray, jintArray, jint);
jlong JN(shardBuild)(JNIEnv *, jclass, jlong, jintArray, jlongArray, jintArray, jintArray, jint, jint, jintArray);
void JN(shardFree)(JNIEnv *, jclass, jlong);
jintArray JN(shardLocalAtoms)(JNIEnv *, jclass, jlong);
jintArray JN(shardOwners)(JNIEnv *, jclass, jlong);
jlong JN(patternBatch)(JNIEnv *, jclass, jlong, jintArray, jlongArray, jintArray, jintArray, jlongArray, jintArray);
jlong JN(rcclCreate)(JNIEnv *, jclass, jbyteArray, jint, jint, jint);

enum { K_INT = 0, K_LONG = 1, K_BYTE = 2 };
static int failures = 0;
static JNIEnv *E;

#define CHECK(c, ...)                                                 \
    do {                                                              \
        if (!(c)) {                                                   \
            fprintf(stderr, "jni_check FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                             \
            fprintf(stderr, "\n");                                    \
            failures++;                                               \
        }                                                             \
    } while (0)

/* after every call: pins released, discipline kept; returns the pending exception class (cleared) */
static const char *settle(const char *what) {
    CHECK(fj_outstanding_pins(E) == 0, "%s: %lld pins outstanding", what, (long long)fj_outstanding_pins(E));
    CHECK(fj_violations(E) == 0, "%s: JNI discipline: %s", what, fj_violation_text(E));
    const char *c = fj_exception_class(E);
    static char cls[160];
    cls[0] = 0;
    if (c) {
        snprintf(cls, sizeof cls, "%s", c);
        fj_exception_clear(E);
    }
    return cls;
}

static jintArray ints(const int32_t *v, int64_t n) { return (jintArray)fj_new_array(E, K_INT, v, n); }
static jlongArray longs(const int64_t *v, int64_t n) { return (jlongArray)fj_new_array(E, K_LONG, v, n); }

/* a small hypergraph: 12 atoms, links 12..17 over the node atoms 0..11 (arity 2..4) */
enum { A = 18, M = 6 };
static const int32_t LA[M] = {12, 13, 14, 15, 16, 17};
static const int64_t OFF[M + 1] = {0, 2, 5, 9, 11, 14, 16};
static const int32_t TG[16] = {0, 1, 1, 2, 3, 3, 4, 5, 6, 6, 7, 8, 9, 10, 10, 11};
static const int32_t TY[M] = {1, 1, 2, 2, 1, 3};

static void check_version_and_nulls(void) {
    jstring v = JN(version)(E, NULL);
    CHECK(v && strncmp((const char *)fj_data(v), "hgx ", 4) == 0, "version");
    settle("version");
    CHECK(JN(lastError)(E, NULL) != NULL, "lastError");
    settle("lastError");
    const char *cls;
    JN(graphInfo)(E, NULL, 0);
    cls = settle("graphInfo(0)");
    CHECK(strcmp(cls, "org/hypergraphdb/HGException") == 0, "graphInfo(0) threw %s", cls);
    JN(bfsInfo)(E, NULL, 0);
    cls = settle("bfsInfo(0)");
    CHECK(strcmp(cls, "org/hypergraphdb/HGException") == 0, "bfsInfo(0) threw %s", cls);
    JN(queryOffsets)(E, NULL, 0);
    cls = settle("queryOffsets(0)");
    CHECK(strcmp(cls, "org/hypergraphdb/HGException") == 0, "queryOffsets(0) threw %s", cls);
    JN(shardInfo)(E, NULL, 0);
    cls = settle("shardInfo(0)");
    CHECK(strcmp(cls, "org/hypergraphdb/HGException") == 0, "shardInfo(0) threw %s", cls);
    JN(seqOffsets)(E, NULL, 0);
    cls = settle("seqOffsets(0)");
    CHECK(strcmp(cls, "org/hypergraphdb/HGException") == 0, "seqOffsets(0) threw %s", cls);
    char bad_id[100] = {0};
    JN(rcclCreate)(E, NULL, (jbyteArray)fj_new_array(E, K_BYTE, bad_id, 100), 2, 0, 0);
    cls = settle("rcclCreate(short id)");
    CHECK(strcmp(cls, "java/lang/IllegalArgumentException") == 0, "rcclCreate threw %s", cls);
}

static void check_snapshot_file(const char *dir) {
    char path[512];
    snprintf(path, sizeof path, "%s/jni_check.hgcsr", dir);
    int8_t handles[A * 8];
    for (int i = 0; i < A * 8; i++) handles[i] = (int8_t)(i * 7 + 3);
    jstring p = (jstring)fj_new_string(E, path);
    JN(snapshotWrite)(E, NULL, p, A, ints(LA, M), longs(OFF, M + 1), ints(TG, 16), ints(TY, M),
                      (jbyteArray)fj_new_array(E, K_BYTE, handles, A * 8), 8);
    const char *cls = settle("snapshotWrite");
    CHECK(cls[0] == 0, "snapshotWrite threw %s: %s", cls, "");
    jlongArray info = JN(snapshotInfo)(E, NULL, p);
    settle("snapshotInfo");
    CHECK(info && fj_length(info) == 5, "snapshotInfo length");
    if (info) {
        const int64_t *v = (const int64_t *)fj_data(info);
        CHECK(v[0] == A && v[1] == M && v[2] == 16 && v[3] == 8, "snapshotInfo %lld %lld %lld %lld", (long long)v[0],
              (long long)v[1], (long long)v[2], (long long)v[3]);
    }
    jbyteArray h = JN(snapshotHandles)(E, NULL, p);
    settle("snapshotHandles");
    CHECK(h && fj_length(h) == A * 8 && memcmp(fj_data(h), handles, A * 8) == 0, "snapshotHandles round trip");
    /* a handle table of the wrong length; an offsets table past its data; a decreasing one */
    JN(snapshotWrite)(E, NULL, p, A, ints(LA, M), longs(OFF, M + 1), ints(TG, 16), ints(TY, M),
                      (jbyteArray)fj_new_array(E, K_BYTE, handles, A * 8 - 1), 8);
    cls = settle("snapshotWrite(short handles)");
    CHECK(strcmp(cls, "java/lang/IllegalArgumentException") == 0, "short handles threw %s", cls);
    int64_t past[M + 1];
    memcpy(past, OFF, sizeof past);
    past[M] = 17;
    JN(snapshotWrite)(E, NULL, p, A, ints(LA, M), longs(past, M + 1), ints(TG, 16), ints(TY, M), NULL, 0);
    cls = settle("snapshotWrite(offsets past data)");
    CHECK(strcmp(cls, "java/lang/IllegalArgumentException") == 0, "offsets past data threw %s", cls);
    int64_t dec[M + 1];
    memcpy(dec, OFF, sizeof dec);
    dec[2] = 1;
    JN(snapshotWrite)(E, NULL, p, A, ints(LA, M), longs(dec, M + 1), ints(TG, 16), ints(TY, M), NULL, 0);
    cls = settle("snapshotWrite(decreasing offsets)");
    CHECK(strcmp(cls, "java/lang/IllegalArgumentException") == 0, "decreasing offsets threw %s", cls);
    JN(snapshotWrite)(E, NULL, NULL, A, ints(LA, M), longs(OFF, M + 1), ints(TG, 16), ints(TY, M), NULL, 0);
    cls = settle("snapshotWrite(null path)");
    CHECK(strcmp(cls, "java/lang/NullPointerException") == 0, "null path threw %s", cls);
    /* OutOfMemoryError at each of the five pins: thrown, every earlier pin released */
    for (int k = 1; k <= 5; k++) {
        fj_inject_oom(E, k);
        JN(snapshotWrite)(E, NULL, p, A, ints(LA, M), longs(OFF, M + 1), ints(TG, 16), ints(TY, M),
                          (jbyteArray)fj_new_array(E, K_BYTE, handles, A * 8), 8);
        fj_inject_oom(E, 0);
        cls = settle("snapshotWrite(oom)");
        CHECK(strcmp(cls, "java/lang/OutOfMemoryError") == 0, "oom at pin %d threw '%s'", k, cls);
    }
}

static void check_partition(void) {
    for (int np = 1; np <= 4; np++) {
        jintArray plan = JN(partitionPlan)(E, NULL, A, ints(LA, M), longs(OFF, M + 1), ints(TG, 16), ints(TY, M), np);
        const char *cls = settle("partitionPlan");
        CHECK(cls[0] == 0 && plan && fj_length(plan) == M, "partitionPlan(%d) threw '%s'", np, cls);
        if (!plan) continue;
        const int32_t *pl = (const int32_t *)fj_data(plan);
        for (int i = 0; i < M; i++) CHECK(pl[i] >= 0 && pl[i] < np, "plan[%d] = %d of %d parts", i, pl[i], np);
        int64_t owned = 0;
        for (int part = 0; part < np; part++) {
            jlong s = JN(shardBuild)(E, NULL, A, ints(LA, M), longs(OFF, M + 1), ints(TG, 16), ints(TY, M), np, part,
                                     plan);
            cls = settle("shardBuild");
            CHECK(cls[0] == 0 && s, "shardBuild(%d/%d) threw '%s'", part, np, cls);
            if (!s) continue;
            jlongArray info = JN(shardInfo)(E, NULL, s);
            settle("shardInfo");
            jintArray l2g = JN(shardLocalAtoms)(E, NULL, s);
            settle("shardLocalAtoms");
            jintArray own = JN(shardOwners)(E, NULL, s);
            settle("shardOwners");
            if (info && l2g && own) {
                const int64_t *v = (const int64_t *)fj_data(info);
                CHECK(fj_length(l2g) == v[0] && fj_length(own) == v[0], "shard tables sized by shardInfo");
                /* per local atom: the owner part of a ghost, -1 for an atom this part owns */
                const int32_t *o = (const int32_t *)fj_data(own);
                for (int64_t i = 0; i < v[0]; i++) {
                    CHECK(o[i] == -1 || (o[i] >= 0 && o[i] < np && o[i] != part), "owner %d on part %d", o[i], part);
                    owned += o[i] == -1;
                }
            }
            JN(shardFree)(E, NULL, s);
            settle("shardFree");
        }
        /* every atom with incidence is owned by exactly one part */
        CHECK(owned == 12, "%d parts own %lld atoms, expected 12", np, (long long)owned);
        /* a plan of the wrong length */
        JN(shardBuild)(E, NULL, A, ints(LA, M), longs(OFF, M + 1), ints(TG, 16), ints(TY, M), np, 0, ints(LA, M - 1));
        cls = settle("shardBuild(short plan)");
        CHECK(strcmp(cls, "java/lang/IllegalArgumentException") == 0, "short plan threw %s", cls);
    }
}

/* argument checks that fire before the engine (so before any GPU): graph rows, pattern batches */
static void check_argument_errors(void) {
    int64_t past[M + 1];
    memcpy(past, OFF, sizeof past);
    past[M] = 99;
    JN(graphCreate)(E, NULL, A, ints(LA, M), longs(past, M + 1), ints(TG, 16), ints(TY, M), 0);
    const char *cls = settle("graphCreate(offsets past data)");
    CHECK(strcmp(cls, "java/lang/IllegalArgumentException") == 0, "graphCreate threw %s", cls);
    JN(graphCreate)(E, NULL, A, ints(LA, M), longs(OFF, M), ints(TG, 16), ints(TY, M), 0);
    cls = settle("graphCreate(short offsets)");
    CHECK(strcmp(cls, "java/lang/IllegalArgumentException") == 0, "graphCreate short offsets threw %s", cls);
    JN(graphCreate)(E, NULL, A, ints(LA, M), longs(OFF, M + 1), ints(TG, 16), ints(TY, M - 2), 0);
    cls = settle("graphCreate(short types)");
    CHECK(strcmp(cls, "java/lang/IllegalArgumentException") == 0, "graphCreate short types threw %s", cls);
    /* a pattern batch of 2 queries whose incidence offsets reach past the anchor array */
    const int32_t ty[2] = {1, -1}, inc[2] = {0, 3}, ho[2] = {0, 0}, pat[1] = {0};
    const int64_t io_bad[3] = {0, 1, 5}, po[3] = {0, 0, 0};
    JN(patternBatch)(E, NULL, 1, ints(ty, 2), longs(io_bad, 3), ints(inc, 2), ints(ho, 2), longs(po, 3), ints(pat, 0));
    cls = settle("patternBatch(offsets past anchors)");
    CHECK(strcmp(cls, "java/lang/IllegalArgumentException") == 0, "patternBatch threw %s", cls);
}

/* Handle tables beyond one Java array: a sparse 300M-atom file with 16-byte handles (4.8 GB of table,
 * config 4's size) read by ranges, the whole-table reader refused; the streamed writer in pieces whose
 * sizes carry partial checksum words, identical to snapshotWrite's file, and its refusals. */
static void check_large_tables(const char *dir) {
    char path[512];
    snprintf(path, sizeof path, "%s/jni_check_big.hgcsr", dir);
    const int64_t BA = 300000000, HB = 16;
    unsigned char hdr[64] = {0};
    memcpy(hdr, "HGXCSR1", 8);
    const uint32_t ver = 2, flags = 2, hb32 = (uint32_t)HB;
    memcpy(hdr + 8, &ver, 4);
    memcpy(hdr + 12, &flags, 4);
    memcpy(hdr + 16, &BA, 8);
    memcpy(hdr + 40, &hb32, 4);
    FILE *f = fopen(path, "wb");
    CHECK(f != NULL, "create %s", path);
    if (!f) return;
    fwrite(hdr, 1, 64, f);
    const long total = (long)(((128 + BA * HB + 63) / 64) * 64);   /* handles at 128 (hgx_file.hip layout) */
    CHECK(fseek(f, total - 1, SEEK_SET) == 0 && fputc(0, f) == 0, "extend the file (sparse)");
    fclose(f);
    jstring p = (jstring)fj_new_string(E, path);
    JN(snapshotHandles)(E, NULL, p);
    const char *cls = settle("snapshotHandles(4.8 GB)");
    CHECK(strcmp(cls, "java/lang/UnsupportedOperationException") == 0, "whole 4.8 GB table threw '%s'", cls);
    const int64_t firsts[3] = {0, BA / 2, BA - 1000};
    for (int i = 0; i < 3; i++) {
        jbyteArray r = JN(snapshotHandlesRange)(E, NULL, p, firsts[i], 1000);
        cls = settle("snapshotHandlesRange");
        CHECK(cls[0] == 0 && r && fj_length(r) == 1000 * HB, "range at %lld threw '%s'", (long long)firsts[i], cls);
    }
    JN(snapshotHandlesRange)(E, NULL, p, BA - 10, 11);
    cls = settle("snapshotHandlesRange(past the end)");
    CHECK(strcmp(cls, "java/lang/IllegalArgumentException") == 0, "range past the end threw '%s'", cls);
    JN(snapshotVerify)(E, NULL, p);   /* the synthetic header carries no checksum */
    cls = settle("snapshotVerify(synthetic)");
    CHECK(strcmp(cls, "org/hypergraphdb/HGException") == 0, "verify threw '%s'", cls);
    remove(path);
    /* streamed writer == snapshotWrite, pieces of 1, 5 and A - 6 four-byte handles */
    char ref[512], out[512];
    snprintf(ref, sizeof ref, "%s/jni_check_ref.hgcsr", dir);
    snprintf(out, sizeof out, "%s/jni_check_stream.hgcsr", dir);
    int8_t handles[A * 4];
    for (int i = 0; i < A * 4; i++) handles[i] = (int8_t)(i * 11 + 1);
    jstring pr = (jstring)fj_new_string(E, ref), po = (jstring)fj_new_string(E, out);
    JN(snapshotWrite)(E, NULL, pr, A, ints(LA, M), longs(OFF, M + 1), ints(TG, 16), ints(TY, M),
                      (jbyteArray)fj_new_array(E, K_BYTE, handles, A * 4), 4);
    settle("snapshotWrite(ref)");
    jlong w = JN(snapshotWriterBegin)(E, NULL, po, A, ints(LA, M), longs(OFF, M + 1), ints(TG, 16), ints(TY, M), 4);
    cls = settle("snapshotWriterBegin");
    CHECK(cls[0] == 0 && w != 0, "writer begin threw '%s'", cls);
    const int cuts[4] = {0, 1, 6, A};
    for (int i = 0; i < 3; i++) {
        JN(snapshotWriterHandles)(E, NULL, w, (jbyteArray)fj_new_array(E, K_BYTE, handles + 4 * cuts[i],
                                                                    4 * (cuts[i + 1] - cuts[i])), 4);
        cls = settle("snapshotWriterHandles");
        CHECK(cls[0] == 0, "writer piece %d threw '%s'", i, cls);
    }
    JN(snapshotWriterEnd)(E, NULL, w);
    settle("snapshotWriterEnd");
    FILE *a = fopen(ref, "rb"), *b = fopen(out, "rb");
    CHECK(a && b, "open written files");
    if (a && b) {
        int same = 1, ca, cb;
        do {
            ca = fgetc(a);
            cb = fgetc(b);
            same &= ca == cb;
        } while (ca != EOF && cb != EOF);
        CHECK(same, "streamed file differs from snapshotWrite's");
    }
    if (a) fclose(a);
    if (b) fclose(b);
    JN(snapshotVerify)(E, NULL, po);
    cls = settle("snapshotVerify(streamed)");
    CHECK(cls[0] == 0, "verify of the streamed file threw '%s'", cls);
    /* a short table: end refuses (and frees the writer); half a handle: refused; abort */
    w = JN(snapshotWriterBegin)(E, NULL, po, A, ints(LA, M), longs(OFF, M + 1), ints(TG, 16), ints(TY, M), 4);
    settle("snapshotWriterBegin(2)");
    JN(snapshotWriterHandles)(E, NULL, w, (jbyteArray)fj_new_array(E, K_BYTE, handles, 6), 4);
    cls = settle("snapshotWriterHandles(half a handle)");
    CHECK(strcmp(cls, "java/lang/IllegalArgumentException") == 0, "half a handle threw '%s'", cls);
    JN(snapshotWriterHandles)(E, NULL, w, (jbyteArray)fj_new_array(E, K_BYTE, handles, 8), 4);
    settle("snapshotWriterHandles(2 of A)");
    JN(snapshotWriterEnd)(E, NULL, w);
    cls = settle("snapshotWriterEnd(short)");
    CHECK(strcmp(cls, "org/hypergraphdb/HGException") == 0, "short table end threw '%s'", cls);
    w = JN(snapshotWriterBegin)(E, NULL, po, A, ints(LA, M), longs(OFF, M + 1), ints(TG, 16), ints(TY, M), 4);
    settle("snapshotWriterBegin(3)");
    JN(snapshotWriterAbort)(E, NULL, w);
    settle("snapshotWriterAbort");
    remove(ref);
    remove(out);
}

int main(int argc, char **argv) {
    const char *dir = argc > 1 ? argv[1] : ".";
    E = fj_env_new();
    check_version_and_nulls();
    check_snapshot_file(dir);
    check_large_tables(dir);
    check_partition();
    check_argument_errors();
    fj_env_free(E);
    if (failures) {
        fprintf(stderr, "jni_check: %d failures\n", failures);
        return 1;
    }
    printf("jni_check: all checks passed\n");
    return 0;
}
