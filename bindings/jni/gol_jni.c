/* gol_jni.c -- JNI glue of gameoflife.GolNative (GolNative.scala) over the
 * C ABI of libgol (include/gol.h): what a JVM backend worker binds to drive
 * the generation step on a GPU instead of the cell actors
 * (CellActor.scala:10-102, NextStateCellGathererActor.scala:21-60, driven by
 * BoardCreator.scala:113-116's NextStep tick).
 *
 * Status: syntax-checked in the CPU suite against bindings/jni/jni_min/jni.h
 * (tests/test_jni_glue.py), never run in a JVM -- the image has no JDK.
 * Build for a JVM:
 *   gcc -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *       bindings/jni/gol_jni.c -Lakka-game-of-life_amd/lib -lgol \
 *       -Wl,-rpath,$PWD/akka-game-of-life_amd/lib -o libgol_jni.so
 *
 * Conventions: a context handle is a jlong; every method returns the gol_*
 * status code (0 = ok) and GolNative.check turns a non-zero one into an
 * exception carrying gol_last_error -- Akka's supervisor then restarts the
 * worker (BoardCreator.scala:42-45).  Methods that return a value return
 * the negated status code on failure.  Host buffers are direct NIO buffers
 * in native byte order; their capacities are checked where the C call
 * takes a size. */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>

#include "gol.h"

#define CTX(h) ((gol_ctx*)(intptr_t)(h))

/* Address and capacity (in the buffer's own elements) of a direct buffer;
 * NULL for a null or non-direct buffer. */
static void* buf_addr(JNIEnv* env, jobject buf, jlong* capacity) {
    if (capacity) *capacity = 0;
    if (!buf) return NULL;
    void* p = (*env)->GetDirectBufferAddress(env, buf);
    if (p && capacity) *capacity = (*env)->GetDirectBufferCapacity(env, buf);
    return p;
}

/* Refuse a libgol built for another ABI: version 2 changed the state hash
 * of row-major boards, so hashes logged by a version-1 library differ. */
JNIEXPORT jint JNICALL JNI_OnLoad(JavaVM* vm, void* reserved) {
    (void)vm;
    (void)reserved;
    return gol_abi_version() == GOL_ABI_VERSION ? JNI_VERSION_1_8 : JNI_ERR;
}

/* visWidth / visHeight: GOL_REF_CLIPPED's visible extents w and h of a
 * (w+1) x (h+1) board (0 = width-1 / height-1, the reference's geometry).
 * Throws IllegalStateException (gol_last_error) and returns 0 on failure. */
JNIEXPORT jlong JNICALL Java_gameoflife_GolNative_create(JNIEnv* env, jclass cls, jlong width, jlong height,
                                                         jlong row0, jlong rows, jint topology, jint birth,
                                                         jint survive, jint device, jlong visWidth,
                                                         jlong visHeight) {
    (void)cls;
    gol_config cfg = {0};
    cfg.width = width;
    cfg.height = height;
    cfg.row0 = row0;
    cfg.rows = rows;
    cfg.topology = topology;
    cfg.birth_mask = (uint32_t)birth;
    cfg.survive_mask = (uint32_t)survive;
    cfg.device = device;
    cfg.vis_width = visWidth;
    cfg.vis_height = visHeight;
    gol_ctx* ctx = NULL;
    if (gol_create(&ctx, &cfg) != GOL_OK) {
        (*env)->ThrowNew(env, (*env)->FindClass(env, "java/lang/IllegalStateException"), gol_last_error(NULL));
        return 0;
    }
    return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNICALL Java_gameoflife_GolNative_destroy(JNIEnv* env, jclass cls, jlong h) {
    (void)env;
    (void)cls;
    gol_destroy(CTX(h));
}

JNIEXPORT jstring JNICALL Java_gameoflife_GolNative_lastError(JNIEnv* env, jclass cls, jlong h) {
    (void)cls;
    return (*env)->NewStringUTF(env, gol_last_error(CTX(h)));
}

JNIEXPORT jint JNICALL Java_gameoflife_GolNative_seed(JNIEnv* env, jclass cls, jlong h, jlong seed) {
    (void)env;
    (void)cls;
    return gol_seed(CTX(h), (uint64_t)seed);
}

/* packed: a direct IntBuffer of the shard's rows, wordsPerRow words apart. */
JNIEXPORT jint JNICALL Java_gameoflife_GolNative_load(JNIEnv* env, jclass cls, jlong h, jobject packed,
                                                      jlong wordsPerRow) {
    (void)cls;
    const uint32_t* p = (const uint32_t*)buf_addr(env, packed, NULL);
    return p ? gol_load(CTX(h), p, wordsPerRow) : GOL_EINVAL;
}

/* hashes: a direct LongBuffer, or null; gol_step_ex refuses (GOL_EINVAL,
 * nothing advanced) when it holds fewer than `gens` entries. */
JNIEXPORT jint JNICALL Java_gameoflife_GolNative_step(JNIEnv* env, jclass cls, jlong h, jint gens,
                                                      jobject hashes) {
    (void)cls;
    if (gens < 0) return GOL_EINVAL;
    jlong cap = 0;
    uint64_t* out = (uint64_t*)buf_addr(env, hashes, &cap);
    if (hashes && !out) return GOL_EINVAL;
    return gol_step_ex(CTX(h), (uint32_t)gens, out, (size_t)cap);
}

/* The context's epoch, or the negated status code. */
JNIEXPORT jlong JNICALL Java_gameoflife_GolNative_epoch(JNIEnv* env, jclass cls, jlong h) {
    (void)env;
    (void)cls;
    uint64_t e = 0;
    const int rc = gol_epoch(CTX(h), &e);
    return rc ? -(jlong)rc : (jlong)e;
}

/* out: a direct LongBuffer of >= 1 entry; receives the shard's state hash
 * (DESIGN.md "State hash": shard partials sum, mod 2^64, to the board's). */
JNIEXPORT jint JNICALL Java_gameoflife_GolNative_hash(JNIEnv* env, jclass cls, jlong h, jobject out) {
    (void)cls;
    jlong cap = 0;
    uint64_t* p = (uint64_t*)buf_addr(env, out, &cap);
    return p && cap >= 1 ? gol_hash(CTX(h), p) : GOL_EINVAL;
}

/* packed: a direct IntBuffer of the shard's rows x wordsPerRow words. */
JNIEXPORT jint JNICALL Java_gameoflife_GolNative_snapshot(JNIEnv* env, jclass cls, jlong h, jobject packed,
                                                          jlong wordsPerRow) {
    (void)cls;
    uint32_t* p = (uint32_t*)buf_addr(env, packed, NULL);
    return p ? gol_snapshot(CTX(h), p, wordsPerRow) : GOL_EINVAL;
}

/* Background dump every so many epochs: `packed` a direct IntBuffer over
 * page-locked memory (hostAlloc); do not read it before snapshotWait. */
JNIEXPORT jint JNICALL Java_gameoflife_GolNative_snapshotAsync(JNIEnv* env, jclass cls, jlong h, jobject packed,
                                                               jlong wordsPerRow) {
    (void)cls;
    uint32_t* p = (uint32_t*)buf_addr(env, packed, NULL);
    return p ? gol_snapshot_async(CTX(h), p, wordsPerRow) : GOL_EINVAL;
}

/* The snapshot's epoch, or the negated status code. */
JNIEXPORT jlong JNICALL Java_gameoflife_GolNative_snapshotWait(JNIEnv* env, jclass cls, jlong h) {
    (void)env;
    (void)cls;
    uint64_t epoch = 0;
    const int rc = gol_snapshot_wait(CTX(h), &epoch);
    return rc ? -(jlong)rc : (jlong)epoch;
}

/* Non-blocking poll of a background snapshot: 1 landed, 0 in flight,
 * negative: the negated status code. */
JNIEXPORT jint JNICALL Java_gameoflife_GolNative_snapshotQuery(JNIEnv* env, jclass cls, jlong h) {
    (void)env;
    (void)cls;
    int landed = 0;
    const int rc = gol_snapshot_query(CTX(h), &landed);
    return rc ? -rc : landed;
}

/* Page-locked host memory as a direct ByteBuffer (freed with hostFree). */
JNIEXPORT jobject JNICALL Java_gameoflife_GolNative_hostAlloc(JNIEnv* env, jclass cls, jlong bytes) {
    (void)cls;
    void* p = NULL;
    if (bytes <= 0 || gol_host_alloc((size_t)bytes, &p) != GOL_OK) return NULL;
    return (*env)->NewDirectByteBuffer(env, p, bytes);
}

JNIEXPORT void JNICALL Java_gameoflife_GolNative_hostFree(JNIEnv* env, jclass cls, jobject buf) {
    (void)cls;
    gol_host_free(buf_addr(env, buf, NULL));
}

/* The cell (x, y) of this shard: 0 or 1, or the negated status code. */
JNIEXPORT jint JNICALL Java_gameoflife_GolNative_getCell(JNIEnv* env, jclass cls, jlong h, jlong x, jlong y) {
    (void)env;
    (void)cls;
    int state = 0;
    const int rc = gol_get_cell(CTX(h), x, y, &state);
    return rc ? -rc : state;
}

/* Bytes a checkpoint of this shard takes, or the negated status code. */
JNIEXPORT jlong JNICALL Java_gameoflife_GolNative_checkpointBytes(JNIEnv* env, jclass cls, jlong h) {
    (void)env;
    (void)cls;
    size_t bytes = 0;
    const int rc = gol_checkpoint_bytes(CTX(h), &bytes);
    return rc ? -(jlong)rc : (jlong)bytes;
}

/* out: a direct ByteBuffer of >= checkpointBytes bytes. */
JNIEXPORT jint JNICALL Java_gameoflife_GolNative_checkpoint(JNIEnv* env, jclass cls, jlong h, jobject out) {
    (void)cls;
    jlong cap = 0;
    void* p = buf_addr(env, out, &cap);
    return p ? gol_checkpoint(CTX(h), p, (size_t)cap) : GOL_EINVAL;
}

/* As checkpoint, in the background (finished by snapshotWait). */
JNIEXPORT jint JNICALL Java_gameoflife_GolNative_checkpointAsync(JNIEnv* env, jclass cls, jlong h, jobject out) {
    (void)cls;
    jlong cap = 0;
    void* p = buf_addr(env, out, &cap);
    return p ? gol_checkpoint_async(CTX(h), p, (size_t)cap) : GOL_EINVAL;
}

/* in: a direct ByteBuffer holding a checkpoint of this shard's rows. */
JNIEXPORT jint JNICALL Java_gameoflife_GolNative_restore(JNIEnv* env, jclass cls, jlong h, jobject in) {
    (void)cls;
    jlong cap = 0;
    const void* p = buf_addr(env, in, &cap);
    return p ? gol_restore(CTX(h), p, (size_t)cap) : GOL_EINVAL;
}

/* A restored block stepped alone through its light cone (BoardCreator.scala:
 * 120-154's re-deploy): above / below direct
 * IntBuffers of `gens` rows each, wordsPerRow apart; hashes a direct
 * LongBuffer of >= gens entries, or null. */
JNIEXPORT jint JNICALL Java_gameoflife_GolNative_replay(JNIEnv* env, jclass cls, jlong h, jint gens, jobject above,
                                                        jobject below, jlong wordsPerRow, jobject hashes) {
    (void)cls;
    jlong cap_a = 0, cap_b = 0, cap_h = 0;
    const uint32_t* a = (const uint32_t*)buf_addr(env, above, &cap_a);
    const uint32_t* b = (const uint32_t*)buf_addr(env, below, &cap_b);
    uint64_t* out = (uint64_t*)buf_addr(env, hashes, &cap_h);
    if (gens < 0 || !a || !b || (hashes && (!out || cap_h < gens))) return GOL_EINVAL;
    if (cap_a < (jlong)gens * wordsPerRow || cap_b < (jlong)gens * wordsPerRow) return GOL_EINVAL;
    return gol_replay(CTX(h), (uint32_t)gens, a, b, wordsPerRow, out);
}

/* Rank 0's RCCL unique id (GOL_UNIQUE_ID_BYTES bytes), to ship to the other
 * backends in the deployment message; null on failure. */
JNIEXPORT jbyteArray JNICALL Java_gameoflife_GolNative_commUniqueId(JNIEnv* env, jclass cls) {
    (void)cls;
    uint8_t id[GOL_UNIQUE_ID_BYTES];
    if (gol_comm_unique_id(id) != GOL_OK) return NULL;
    jbyteArray arr = (*env)->NewByteArray(env, GOL_UNIQUE_ID_BYTES);
    if (arr) (*env)->SetByteArrayRegion(env, arr, 0, GOL_UNIQUE_ID_BYTES, (const jbyte*)id);
    return arr;
}

JNIEXPORT jint JNICALL Java_gameoflife_GolNative_commInit(JNIEnv* env, jclass cls, jlong h, jbyteArray id,
                                                          jint rank, jint n) {
    (void)cls;
    if (!id || (*env)->GetArrayLength(env, id) != GOL_UNIQUE_ID_BYTES) return GOL_EINVAL;
    jbyte buf[GOL_UNIQUE_ID_BYTES];
    (*env)->GetByteArrayRegion(env, id, 0, GOL_UNIQUE_ID_BYTES, buf);
    return gol_comm_init(CTX(h), (const uint8_t*)buf, rank, n);
}

JNIEXPORT jint JNICALL Java_gameoflife_GolNative_commAbort(JNIEnv* env, jclass cls, jlong h) {
    (void)env;
    (void)cls;
    return gol_comm_abort(CTX(h));
}

/* Sum (mod 2^64) of `count` u64 over the ring, in place: values a direct
 * LongBuffer of >= count entries (the global hash from shard partials). */
JNIEXPORT jint JNICALL Java_gameoflife_GolNative_commAllreduce(JNIEnv* env, jclass cls, jlong h, jobject values,
                                                               jint count) {
    (void)cls;
    jlong cap = 0;
    uint64_t* p = (uint64_t*)buf_addr(env, values, &cap);
    if (count < 0 || (count > 0 && (!p || cap < count))) return GOL_EINVAL;
    return gol_comm_allreduce_u64(CTX(h), p, (uint32_t)count);
}

/* Rows of rank `rank` of `n`: out a direct LongBuffer of 2 entries (row0, rows). */
JNIEXPORT jint JNICALL Java_gameoflife_GolNative_shardRows(JNIEnv* env, jclass cls, jlong height, jint rank, jint n,
                                                           jobject out) {
    (void)cls;
    jlong cap = 0;
    int64_t* p = (int64_t*)buf_addr(env, out, &cap);
    if (!p || cap < 2) return GOL_EINVAL;
    return gol_shard_rows(height, rank, n, &p[0], &p[1]);
}

JNIEXPORT jint JNICALL Java_gameoflife_GolNative_setTuning(JNIEnv* env, jclass cls, jlong h, jint bandRows,
                                                           jint gensPerPass, jint wordsPerLane) {
    (void)env;
    (void)cls;
    return gol_set_tuning(CTX(h), bandRows, gensPerPass, wordsPerLane);
}

JNIEXPORT jint JNICALL Java_gameoflife_GolNative_profileEnable(JNIEnv* env, jclass cls, jlong h, jboolean on) {
    (void)env;
    (void)cls;
    return gol_profile_enable(CTX(h), on ? 1 : 0);
}

/* out: a direct ByteBuffer (native order) of >= sizeof(gol_profile_stats)
 * = 96 bytes; the fields in gol.h's order, 8 bytes each. */
JNIEXPORT jint JNICALL Java_gameoflife_GolNative_profileStats(JNIEnv* env, jclass cls, jlong h, jobject out) {
    (void)cls;
    jlong cap = 0;
    gol_profile_stats* p = (gol_profile_stats*)buf_addr(env, out, &cap);
    if (!p || cap < (jlong)sizeof(gol_profile_stats)) return GOL_EINVAL;
    return gol_profile_stats_read(CTX(h), p);
}

/* The HIP runtime and RCCL this process's libgol is bound to, to log next to
 * a backend's first hashes. */
JNIEXPORT jstring JNICALL Java_gameoflife_GolNative_runtimeInfo(JNIEnv* env, jclass cls) {
    (void)cls;
    gol_runtime_info ri;
    char buf[1700];
    if (gol_runtime_info_get(&ri) != GOL_OK) return NULL;
    snprintf(buf, sizeof buf, "HIP %d (%s), RCCL %d (%s), libgol %s", (int)ri.hip_runtime_version, ri.hip_library,
             (int)ri.rccl_version, ri.rccl_library, ri.gol_library);
    return (*env)->NewStringUTF(env, buf);
}
