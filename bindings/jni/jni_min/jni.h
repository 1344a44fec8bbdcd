/* jni_min/jni.h -- a minimal JNI declaration subset for SYNTAX-CHECKING
 * bindings/jni/gol_jni.c in the CPU test suite (tests/test_jni_glue.py),
 * where no JDK is installed.  It is NOT the JDK's jni.h: the types and the
 * names and signatures of the JNIEnv functions the glue calls follow the JNI
 * 1.8 specification, but the function table holds only those entries, so
 * its layout is not the JDK's.  A loadable libgol_jni.so must be built
 * against $JAVA_HOME/include. */
#ifndef GOL_JNI_MIN_H
#define GOL_JNI_MIN_H
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_OK 0
#define JNI_ERR (-1)
#define JNI_VERSION_1_8 0x00010008

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef jint jsize;

struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jbyteArray;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;
struct JNIInvokeInterface_;
typedef const struct JNIInvokeInterface_* JavaVM;

struct JNINativeInterface_ {
    jclass (JNICALL* FindClass)(JNIEnv* env, const char* name);
    jint (JNICALL* ThrowNew)(JNIEnv* env, jclass clazz, const char* msg);
    jboolean (JNICALL* ExceptionCheck)(JNIEnv* env);
    jstring (JNICALL* NewStringUTF)(JNIEnv* env, const char* utf);
    jsize (JNICALL* GetArrayLength)(JNIEnv* env, jarray array);
    jbyteArray (JNICALL* NewByteArray)(JNIEnv* env, jsize len);
    void (JNICALL* GetByteArrayRegion)(JNIEnv* env, jbyteArray array, jsize start, jsize len, jbyte* buf);
    void (JNICALL* SetByteArrayRegion)(JNIEnv* env, jbyteArray array, jsize start, jsize len, const jbyte* buf);
    jobject (JNICALL* NewDirectByteBuffer)(JNIEnv* env, void* address, jlong capacity);
    void* (JNICALL* GetDirectBufferAddress)(JNIEnv* env, jobject buf);
    jlong (JNICALL* GetDirectBufferCapacity)(JNIEnv* env, jobject buf);
};

#endif
