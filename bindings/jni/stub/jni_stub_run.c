/* jni_stub_run.c -- runs the JNI glue (bindings/jni/gol_jni.c) without a JVM.
 *
 * The image has no JDK, so this harness plays the JVM's part for the calls a
 * GpuBackendWorker (GolNative.scala) makes: it builds a JNIEnv whose function
 * table (bindings/jni/jni_min/jni.h) backs direct NIO buffers, byte arrays,
 * strings and exceptions with plain C objects, then calls the
 * Java_gameoflife_GolNative_* entry points in the order the worker does --
 * create, seed, step with a hash buffer, hash, background snapshot, the
 * capacity checks, checkpoint and restore into a second context, shard rows,
 * runtime info, profile stats, destroy -- and prints one JSON line that
 * tests/test_gpu_jni_stub.py checks against the CPU oracle.  It exercises the
 * glue's own logic (buffer addressing, capacity checks, status and exception
 * paths) on the GPU; it does not exercise a JVM.
 *
 *   jni_stub_run W H GENS SEED
 */
#include <jni.h>
#include <inttypes.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gol.h"

/* ---- the stub JVM objects ------------------------------------------------ */

enum { K_CLASS = 1, K_STRING, K_BYTES, K_BUFFER };

struct _jobject {
    int kind;
    void* addr;     /* buffer memory, string bytes or array bytes */
    jlong capacity; /* buffers: elements; arrays: length */
};

static struct _jobject g_class = {K_CLASS, NULL, 0};
static char g_thrown[512];

static jobject new_obj(int kind, void* addr, jlong capacity) {
    jobject o = (jobject)calloc(1, sizeof *o);
    o->kind = kind;
    o->addr = addr;
    o->capacity = capacity;
    return o;
}

/* A direct buffer view of `addr`: `capacity` elements (as NIO reports them). */
static jobject direct(void* addr, jlong capacity) { return new_obj(K_BUFFER, addr, capacity); }

static jclass JNICALL s_FindClass(JNIEnv* env, const char* name) {
    (void)env;
    (void)name;
    return &g_class;
}
static jint JNICALL s_ThrowNew(JNIEnv* env, jclass c, const char* msg) {
    (void)env;
    (void)c;
    snprintf(g_thrown, sizeof g_thrown, "%s", msg ? msg : "");
    return 0;
}
static jboolean JNICALL s_ExceptionCheck(JNIEnv* env) {
    (void)env;
    return g_thrown[0] != 0;
}
static jstring JNICALL s_NewStringUTF(JNIEnv* env, const char* utf) {
    (void)env;
    const char* u = utf ? utf : "";
    char* copy = (char*)malloc(strlen(u) + 1);
    memcpy(copy, u, strlen(u) + 1);
    return new_obj(K_STRING, copy, (jlong)strlen(u));
}
static jsize JNICALL s_GetArrayLength(JNIEnv* env, jarray a) {
    (void)env;
    return (jsize)a->capacity;
}
static jbyteArray JNICALL s_NewByteArray(JNIEnv* env, jsize len) {
    (void)env;
    return new_obj(K_BYTES, calloc((size_t)len, 1), len);
}
static void JNICALL s_GetByteArrayRegion(JNIEnv* env, jbyteArray a, jsize start, jsize len, jbyte* buf) {
    (void)env;
    memcpy(buf, (jbyte*)a->addr + start, (size_t)len);
}
static void JNICALL s_SetByteArrayRegion(JNIEnv* env, jbyteArray a, jsize start, jsize len, const jbyte* buf) {
    (void)env;
    memcpy((jbyte*)a->addr + start, buf, (size_t)len);
}
static jobject JNICALL s_NewDirectByteBuffer(JNIEnv* env, void* addr, jlong cap) {
    (void)env;
    return direct(addr, cap);
}
static void* JNICALL s_GetDirectBufferAddress(JNIEnv* env, jobject b) {
    (void)env;
    return b && b->kind == K_BUFFER ? b->addr : NULL;
}
static jlong JNICALL s_GetDirectBufferCapacity(JNIEnv* env, jobject b) {
    (void)env;
    return b && b->kind == K_BUFFER ? b->capacity : -1;
}

static const struct JNINativeInterface_ g_table = {
    s_FindClass,          s_ThrowNew,          s_ExceptionCheck,        s_NewStringUTF,
    s_GetArrayLength,     s_NewByteArray,      s_GetByteArrayRegion,    s_SetByteArrayRegion,
    s_NewDirectByteBuffer, s_GetDirectBufferAddress, s_GetDirectBufferCapacity,
};

/* ---- the glue's entry points (gol_jni.c) --------------------------------- */

jint JNI_OnLoad(JavaVM* vm, void* reserved);
jlong Java_gameoflife_GolNative_create(JNIEnv*, jclass, jlong, jlong, jlong, jlong, jint, jint, jint, jint, jlong,
                                       jlong);
void Java_gameoflife_GolNative_destroy(JNIEnv*, jclass, jlong);
jstring Java_gameoflife_GolNative_lastError(JNIEnv*, jclass, jlong);
jint Java_gameoflife_GolNative_seed(JNIEnv*, jclass, jlong, jlong);
jint Java_gameoflife_GolNative_step(JNIEnv*, jclass, jlong, jint, jobject);
jlong Java_gameoflife_GolNative_epoch(JNIEnv*, jclass, jlong);
jint Java_gameoflife_GolNative_hash(JNIEnv*, jclass, jlong, jobject);
jint Java_gameoflife_GolNative_snapshot(JNIEnv*, jclass, jlong, jobject, jlong);
jint Java_gameoflife_GolNative_snapshotAsync(JNIEnv*, jclass, jlong, jobject, jlong);
jlong Java_gameoflife_GolNative_snapshotWait(JNIEnv*, jclass, jlong);
jobject Java_gameoflife_GolNative_hostAlloc(JNIEnv*, jclass, jlong);
void Java_gameoflife_GolNative_hostFree(JNIEnv*, jclass, jobject);
jint Java_gameoflife_GolNative_getCell(JNIEnv*, jclass, jlong, jlong, jlong);
jlong Java_gameoflife_GolNative_checkpointBytes(JNIEnv*, jclass, jlong);
jint Java_gameoflife_GolNative_checkpoint(JNIEnv*, jclass, jlong, jobject);
jint Java_gameoflife_GolNative_restore(JNIEnv*, jclass, jlong, jobject);
jint Java_gameoflife_GolNative_shardRows(JNIEnv*, jclass, jlong, jint, jint, jobject);
jint Java_gameoflife_GolNative_profileEnable(JNIEnv*, jclass, jlong, jboolean);
jint Java_gameoflife_GolNative_profileStats(JNIEnv*, jclass, jlong, jobject);
jstring Java_gameoflife_GolNative_runtimeInfo(JNIEnv*, jclass);

#define N(x) Java_gameoflife_GolNative_##x

int main(int argc, char** argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s W H GENS SEED\n", argv[0]);
        return 2;
    }
    const jlong W = atoll(argv[1]), H = atoll(argv[2]);
    const jint gens = atoi(argv[3]);
    const jlong seed = strtoll(argv[4], NULL, 0);
    const JNIEnv envp = &g_table;
    JNIEnv* env = (JNIEnv*)&envp;
    jclass cls = &g_class;
    const long words = (long)((W + 31) / 32);
    int fails = 0;
#define EXPECT(cond, what)                                              \
    do {                                                                \
        if (!(cond)) {                                                  \
            fprintf(stderr, "jni_stub_run: %s failed (line %d)\n", what, __LINE__); \
            ++fails;                                                    \
        }                                                               \
    } while (0)

    EXPECT(JNI_OnLoad(NULL, NULL) == JNI_VERSION_1_8, "JNI_OnLoad");

    /* a board that cannot exist: the exception path of create */
    g_thrown[0] = 0;
    EXPECT(N(create)(env, cls, 33, 8, 0, 0, GOL_TORUS, 8, 12, 0, 0, 0) == 0 && g_thrown[0] != 0, "create refuses");
    char thrown[512];
    snprintf(thrown, sizeof thrown, "%s", g_thrown);
    g_thrown[0] = 0;

    const jlong h = N(create)(env, cls, W, H, 0, 0, GOL_TORUS, GOL_RULE_LIFE_BIRTH, GOL_RULE_LIFE_SURVIVE, 0, 0, 0);
    if (!h) {
        fprintf(stderr, "jni_stub_run: create: %s\n", g_thrown);
        return 1;
    }
    EXPECT(N(seed)(env, cls, h, seed) == GOL_OK, "seed");

    /* step with a LongBuffer one entry too small: refused, nothing advanced */
    uint64_t* hashes = (uint64_t*)calloc((size_t)gens + 1, sizeof(uint64_t));
    const jint rc_small = N(step)(env, cls, h, gens, direct(hashes, gens - 1));
    EXPECT(rc_small == GOL_EINVAL && N(epoch)(env, cls, h) == 0, "step capacity check");
    jstring err = N(lastError)(env, cls, h);

    EXPECT(N(profileEnable)(env, cls, h, 1) == GOL_OK, "profileEnable");
    EXPECT(N(step)(env, cls, h, gens, direct(hashes, gens)) == GOL_OK, "step");
    const jlong epoch = N(epoch)(env, cls, h);
    uint64_t final_hash = 0;
    EXPECT(N(hash)(env, cls, h, direct(&final_hash, 1)) == GOL_OK, "hash");
    unsigned char stats[96];
    EXPECT(N(profileStats)(env, cls, h, direct(stats, 95)) == GOL_EINVAL, "profileStats capacity check");
    EXPECT(N(profileStats)(env, cls, h, direct(stats, sizeof stats)) == GOL_OK, "profileStats");
    gol_profile_stats ps;
    memcpy(&ps, stats, sizeof ps);

    /* background snapshot into page-locked memory, as the worker's dump */
    const jlong snap_bytes = (jlong)H * words * 4;
    jobject pinned = N(hostAlloc)(env, cls, snap_bytes);
    EXPECT(pinned != NULL, "hostAlloc");
    uint32_t* snap = pinned ? (uint32_t*)pinned->addr : NULL;
    EXPECT(pinned && N(snapshotAsync)(env, cls, h, direct(snap, H * words), words) == GOL_OK, "snapshotAsync");
    const jlong snap_epoch = N(snapshotWait)(env, cls, h);
    EXPECT(snap_epoch == epoch, "snapshotWait epoch");
    uint64_t cell_sum = 0;
    for (long k = 0; k < H * words; ++k) cell_sum += (uint64_t)__builtin_popcount(snap[k]);
    const jint cell00 = N(getCell)(env, cls, h, 0, 0);
    EXPECT(cell00 == (jint)(snap[0] & 1u), "getCell");

    /* checkpoint into a ByteBuffer, restore into a fresh context, same hash */
    const jlong ck_bytes = N(checkpointBytes)(env, cls, h);
    unsigned char* ck = (unsigned char*)malloc((size_t)ck_bytes);
    EXPECT(N(checkpoint)(env, cls, h, direct(ck, ck_bytes - 1)) == GOL_EINVAL, "checkpoint capacity check");
    EXPECT(N(checkpoint)(env, cls, h, direct(ck, ck_bytes)) == GOL_OK, "checkpoint");
    const jlong h2 = N(create)(env, cls, W, H, 0, 0, GOL_TORUS, GOL_RULE_LIFE_BIRTH, GOL_RULE_LIFE_SURVIVE, 0, 0, 0);
    EXPECT(h2 && N(restore)(env, cls, h2, direct(ck, ck_bytes)) == GOL_OK, "restore");
    uint64_t restored_hash = 0;
    EXPECT(h2 && N(hash)(env, cls, h2, direct(&restored_hash, 1)) == GOL_OK, "hash after restore");
    EXPECT(h2 && N(epoch)(env, cls, h2) == epoch, "epoch after restore");

    int64_t rows3[2] = {0, 0};
    EXPECT(N(shardRows)(env, cls, 10, 2, 3, direct(rows3, 2)) == GOL_OK, "shardRows");
    jstring info = N(runtimeInfo)(env, cls);

    printf("{\"width\": %" PRId64 ", \"height\": %" PRId64 ", \"generations\": %d, \"epoch\": %" PRId64
           ", \"hashes\": [",
           (int64_t)W, (int64_t)H, gens, (int64_t)epoch);
    for (jint k = 0; k < gens; ++k) printf("%s\"%" PRIu64 "\"", k ? ", " : "", hashes[k]);
    printf("], \"final_hash\": \"%" PRIu64 "\", \"restored_hash\": \"%" PRIu64 "\", \"snapshot_epoch\": %" PRId64
           ", \"live_cells\": %" PRIu64 ", \"shard_rows_2_of_3\": [%" PRId64 ", %" PRId64 "], \"launches\": %" PRIu64
           ", \"generations_profiled\": %" PRIu64 ", \"step_capacity_rc\": %d",
           final_hash, restored_hash, (int64_t)snap_epoch, cell_sum, rows3[0], rows3[1], ps.launches,
           ps.generations, rc_small);
    printf(", \"create_refused\": \"");
    for (const char* c = thrown; *c; ++c) putchar(*c == '"' || *c == '\\' ? '\'' : *c);
    printf("\", \"step_capacity_error\": \"");
    for (const char* c = err ? (const char*)err->addr : ""; *c; ++c) putchar(*c == '"' || *c == '\\' ? '\'' : *c);
    printf("\", \"runtime\": \"");
    for (const char* c = info ? (const char*)info->addr : ""; *c; ++c) putchar(*c == '"' || *c == '\\' ? '\'' : *c);
    printf("\", \"fails\": %d}\n", fails);

    if (pinned) N(hostFree)(env, cls, pinned);
    if (h2) N(destroy)(env, cls, h2);
    N(destroy)(env, cls, h);
    free(ck);
    free(hashes);
    return fails ? 1 : 0;
}
