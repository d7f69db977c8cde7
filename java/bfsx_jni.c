/*
 * bfsx_jni.c -- JNI forwards of it.unitn.bd.bfs.Bfsx (java/it/unitn/bd/bfs/Bfsx.java) onto the C-ABI of
 * libbfsx.so (include/bfsx.h).  Every native method is a one-call forward: arguments pass through,
 * results land in caller-allocated direct ByteBuffers, a negative BFSX_E_* code becomes the Java
 * exception the reference's code path throws for the same input (see Bfsx.java).
 *
 * Build (java/Makefile): gcc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux
 *   -I../include bfsx_jni.c -L../bfs-with-mapreduce_amd -lbfsx -o libbfsx_jni.so
 * Not compiled in this repository's image (no JDK, so no jni.h).
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

#include "bfsx.h"

#define H(x) ((void *)(intptr_t)(x))
#define J(p) ((jlong)(intptr_t)(p))

static void throw_for(JNIEnv *env, int rc) {
    const char *cls = rc == BFSX_E_IO      ? "java/io/IOException"
                      : rc == BFSX_E_PARSE ? "java/lang/NumberFormatException"
                      : rc == BFSX_E_RANGE ? "java/lang/NullPointerException"
                                           : "java/lang/IllegalStateException";
    jclass c = (*env)->FindClass(env, cls);
    if (c) (*env)->ThrowNew(env, c, bfsx_last_error());
}

/* 1 when rc is an error (the exception is pending: the caller returns at once) */
static int failed(JNIEnv *env, int rc) {
    if (rc >= 0) return 0;
    throw_for(env, rc);
    return 1;
}

/* address of a direct buffer holding at least `bytes`, or NULL (IllegalArgumentException pending) */
static void *direct(JNIEnv *env, jobject buf, jlong bytes) {
    if (!buf) return NULL;
    void *p = (*env)->GetDirectBufferAddress(env, buf);
    if (!p || (*env)->GetDirectBufferCapacity(env, buf) < bytes) {
        jclass c = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
        if (c) (*env)->ThrowNew(env, c, "need a direct ByteBuffer of the graph's size");
        return NULL;
    }
    return p;
}

/* host copies of two int[] tuple arrays as uint32 (ids are non-negative Java ints) */
static int tuples(JNIEnv *env, jintArray u, jintArray v, uint32_t **uu, uint32_t **vv, jsize *m) {
    *m = (*env)->GetArrayLength(env, u);
    if ((*env)->GetArrayLength(env, v) != *m) return BFSX_E_ARG;
    *uu = (uint32_t *)malloc((size_t)(*m > 0 ? *m : 1) * sizeof(uint32_t));
    *vv = (uint32_t *)malloc((size_t)(*m > 0 ? *m : 1) * sizeof(uint32_t));
    if (!*uu || !*vv) {
        free(*uu);
        free(*vv);
        return BFSX_E_OOM;
    }
    (*env)->GetIntArrayRegion(env, u, 0, *m, (jint *)*uu);
    (*env)->GetIntArrayRegion(env, v, 0, *m, (jint *)*vv);
    return BFSX_OK;
}

JNIEXPORT jlong JNICALL Java_it_unitn_bd_bfs_Bfsx_init(JNIEnv *env, jclass cls, jint device) {
    bfsx_ctx *ctx = NULL;
    return failed(env, bfsx_init(device, &ctx)) ? 0 : J(ctx);
}

JNIEXPORT jlong JNICALL Java_it_unitn_bd_bfs_Bfsx_initGroup(JNIEnv *env, jclass cls, jint nranks) {
    bfsx_ctx *ctx = NULL;
    return failed(env, bfsx_init_group(nranks, &ctx)) ? 0 : J(ctx);
}

JNIEXPORT jint JNICALL Java_it_unitn_bd_bfs_Bfsx_groupSize(JNIEnv *env, jclass cls, jlong ctx) {
    const int n = bfsx_group_size(H(ctx));
    return failed(env, n) ? 0 : n;
}

JNIEXPORT void JNICALL Java_it_unitn_bd_bfs_Bfsx_setOption(JNIEnv *env, jclass cls, jlong ctx, jstring key,
                                                          jstring value) {
    const char *k = (*env)->GetStringUTFChars(env, key, NULL);
    const char *v = (*env)->GetStringUTFChars(env, value, NULL);
    const int rc = bfsx_set_option(H(ctx), k, v);
    (*env)->ReleaseStringUTFChars(env, key, k);
    (*env)->ReleaseStringUTFChars(env, value, v);
    failed(env, rc);
}

JNIEXPORT void JNICALL Java_it_unitn_bd_bfs_Bfsx_finalizeContext(JNIEnv *env, jclass cls, jlong ctx) {
    bfsx_finalize(H(ctx));
}

JNIEXPORT jlong JNICALL Java_it_unitn_bd_bfs_Bfsx_loadAlgs4(JNIEnv *env, jclass cls, jlong ctx, jstring path) {
    const char *p = (*env)->GetStringUTFChars(env, path, NULL);
    bfsx_graph *g = NULL;
    const int rc = bfsx_graph_load_algs4(H(ctx), p, &g);
    (*env)->ReleaseStringUTFChars(env, path, p);
    return failed(env, rc) ? 0 : J(g);
}

JNIEXPORT jlong JNICALL Java_it_unitn_bd_bfs_Bfsx_fromEdges(JNIEnv *env, jclass cls, jlong ctx, jlong nv,
                                                           jintArray u, jintArray v) {
    uint32_t *uu, *vv;
    jsize m;
    int rc = tuples(env, u, v, &uu, &vv, &m);
    if (failed(env, rc)) return 0;
    bfsx_graph *g = NULL;
    rc = bfsx_graph_from_edges(H(ctx), nv, uu, vv, m, &g);
    free(uu);
    free(vv);
    return failed(env, rc) ? 0 : J(g);
}

JNIEXPORT jlong JNICALL Java_it_unitn_bd_bfs_Bfsx_nv(JNIEnv *env, jclass cls, jlong g) { return bfsx_graph_nv(H(g)); }

JNIEXPORT jlong JNICALL Java_it_unitn_bd_bfs_Bfsx_nnz(JNIEnv *env, jclass cls, jlong g) { return bfsx_graph_nnz(H(g)); }

JNIEXPORT void JNICALL Java_it_unitn_bd_bfs_Bfsx_csr(JNIEnv *env, jclass cls, jlong g, jobject row_off, jobject col) {
    const jlong nv = bfsx_graph_nv(H(g)), nnz = bfsx_graph_nnz(H(g));
    int64_t *o = (int64_t *)direct(env, row_off, (nv + 1) * 8);
    if (row_off && !o) return;
    uint32_t *c = (uint32_t *)direct(env, col, nnz * 4);
    if (col && !c) return;
    failed(env, bfsx_graph_csr(H(g), o, c));
}

JNIEXPORT void JNICALL Java_it_unitn_bd_bfs_Bfsx_free(JNIEnv *env, jclass cls, jlong g) { bfsx_graph_free(H(g)); }

JNIEXPORT jint JNICALL Java_it_unitn_bd_bfs_Bfsx_bfs(JNIEnv *env, jclass cls, jlong g, jlong source, jobject dist,
                                                    jobject parent) {
    const jlong nv = bfsx_graph_nv(H(g));
    int32_t *d = (int32_t *)direct(env, dist, nv * 4);
    if (dist && !d) return -1;
    int64_t *p = (int64_t *)direct(env, parent, nv * 8);
    if (parent && !p) return -1;
    bfsx_stats st;
    return failed(env, bfsx_bfs(H(g), source, d, p, &st)) ? -1 : st.levels;
}

JNIEXPORT jdoubleArray JNICALL Java_it_unitn_bd_bfs_Bfsx_levelTimesMs(JNIEnv *env, jclass cls, jlong g) {
    /* passes of one BFS: ecc(source) + 1, unknown up front -- grow until the copy is not truncated */
    int cap = 4096, k = 0;
    double *buf = NULL;
    for (;;) {
        double *nb = (double *)realloc(buf, (size_t)cap * sizeof(double));
        if (!nb) {
            free(buf);
            throw_for(env, BFSX_E_OOM);
            return NULL;
        }
        buf = nb;
        k = bfsx_level_times(H(g), buf, cap);
        if (k < cap) break;
        cap *= 2;
    }
    jdoubleArray out = NULL;
    if (!failed(env, k)) {
        out = (*env)->NewDoubleArray(env, k);
        if (out) (*env)->SetDoubleArrayRegion(env, out, 0, k, buf);
    }
    free(buf);
    return out;
}

JNIEXPORT jlong JNICALL Java_it_unitn_bd_bfs_Bfsx_validate(JNIEnv *env, jclass cls, jlong g) {
    int64_t errors = 0;
    return failed(env, bfsx_validate(H(g), -1, &errors, NULL, NULL, NULL)) ? -1 : errors;
}

JNIEXPORT jbyteArray JNICALL Java_it_unitn_bd_bfs_Bfsx_commUniqueId(JNIEnv *env, jclass cls) {
    uint8_t id[BFSX_COMM_ID_BYTES];
    if (failed(env, bfsx_comm_unique_id(id))) return NULL;
    jbyteArray out = (*env)->NewByteArray(env, BFSX_COMM_ID_BYTES);
    if (out) (*env)->SetByteArrayRegion(env, out, 0, BFSX_COMM_ID_BYTES, (const jbyte *)id);
    return out;
}

JNIEXPORT void JNICALL Java_it_unitn_bd_bfs_Bfsx_commTimes(JNIEnv *env, jclass cls, jlong g, jdoubleArray ms,
                                                          jlongArray calls) {
    double m[4];
    int64_t c[4];
    if ((*env)->GetArrayLength(env, ms) < 4 || (*env)->GetArrayLength(env, calls) < 4) {
        throw_for(env, BFSX_E_ARG);
        return;
    }
    if (failed(env, bfsx_comm_times(H(g), m, c))) return;
    jlong cl[4];
    for (int k = 0; k < 4; k++) cl[k] = (jlong)c[k];
    (*env)->SetDoubleArrayRegion(env, ms, 0, 4, m);
    (*env)->SetLongArrayRegion(env, calls, 0, 4, cl);
}

JNIEXPORT void JNICALL Java_it_unitn_bd_bfs_Bfsx_commInit(JNIEnv *env, jclass cls, jlong ctx, jint rank, jint nranks,
                                                         jbyteArray id) {
    uint8_t buf[BFSX_COMM_ID_BYTES];
    if ((*env)->GetArrayLength(env, id) != BFSX_COMM_ID_BYTES) {
        throw_for(env, BFSX_E_ARG);
        return;
    }
    (*env)->GetByteArrayRegion(env, id, 0, BFSX_COMM_ID_BYTES, (jbyte *)buf);
    failed(env, bfsx_comm_init(H(ctx), rank, nranks, buf));
}

JNIEXPORT jlong JNICALL Java_it_unitn_bd_bfs_Bfsx_distKronecker(JNIEnv *env, jclass cls, jlong ctx, jint scale,
                                                               jint edgefactor, jlong seed, jint rank, jint nranks) {
    bfsx_graph *g = NULL;
    return failed(env, bfsx_dist_graph_kronecker(H(ctx), scale, edgefactor, (uint64_t)seed, rank, nranks, &g)) ? 0
                                                                                                              : J(g);
}

JNIEXPORT jlong JNICALL Java_it_unitn_bd_bfs_Bfsx_distFromEdges(JNIEnv *env, jclass cls, jlong ctx, jlong nv,
                                                               jintArray u, jintArray v, jint rank, jint nranks) {
    uint32_t *uu, *vv;
    jsize m;
    int rc = tuples(env, u, v, &uu, &vv, &m);
    if (failed(env, rc)) return 0;
    bfsx_graph *g = NULL;
    rc = bfsx_dist_graph_from_edges(H(ctx), nv, uu, vv, m, rank, nranks, &g);
    free(uu);
    free(vv);
    return failed(env, rc) ? 0 : J(g);
}

JNIEXPORT jint JNICALL Java_it_unitn_bd_bfs_Bfsx_distBfs(JNIEnv *env, jclass cls, jlong g, jlong source) {
    bfsx_stats st;
    return failed(env, bfsx_dist_bfs(H(g), source, &st)) ? -1 : st.levels;
}

JNIEXPORT void JNICALL Java_it_unitn_bd_bfs_Bfsx_result(JNIEnv *env, jclass cls, jlong g, jobject dist,
                                                       jobject parent) {
    const jlong nv = bfsx_graph_nv(H(g));
    int32_t *d = (int32_t *)direct(env, dist, nv * 4);
    if (dist && !d) return;
    int64_t *p = (int64_t *)direct(env, parent, nv * 8);
    if (parent && !p) return;
    failed(env, bfsx_result(H(g), d, p));
}

JNIEXPORT jlongArray JNICALL Java_it_unitn_bd_bfs_Bfsx_partition(JNIEnv *env, jclass cls, jlong g) {
    int64_t a[6] = {0, 0, 0, 0, 0, 0};
    int32_t rank = 0, nranks = 1;
    if (failed(env, bfsx_graph_partition(H(g), &a[0], &a[1], &a[2], &a[3], &rank, &nranks))) return NULL;
    a[4] = rank;
    a[5] = nranks;
    jlongArray out = (*env)->NewLongArray(env, 6);
    if (out) (*env)->SetLongArrayRegion(env, out, 0, 6, (const jlong *)a);
    return out;
}
