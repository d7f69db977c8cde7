package it.unitn.bd.bfs;

import java.io.IOException;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;

/**
 * JNI mirror of the C-ABI in include/bfsx.h (libbfsx.so), through the forwards in java/bfsx_jni.c
 * (libbfsx_jni.so).  Handles are the native pointers as longs.  Result arrays are direct ByteBuffers in
 * native byte order, so the library writes them without a JNI array copy.
 *
 * Error mapping (the exceptions the reference's code path throws for the same input):
 *   BFSX_E_IO    -> IOException                (GraphFileUtil.java:46 FileInputStream)
 *   BFSX_E_PARSE -> NumberFormatException      (GraphFileUtil.java:48,62-63 Integer.parseInt)
 *   BFSX_E_RANGE -> NullPointerException       (GraphFileUtil.java:64-65 vertices.get(id) for id outside [0,V))
 *   anything else -> IllegalStateException     (device / communicator failures; the reference has none)
 *
 * Not compiled in this repository's image (it has no JDK): build with java/Makefile.
 */
public final class Bfsx {

    static {
        System.loadLibrary("bfsx_jni"); // libbfsx_jni.so, linked against libbfsx.so
    }

    /** BFSX_DIR_* of include/bfsx.h (level records). */
    public static final int DIR_TOPDOWN = 1, DIR_BOTTOMUP = 2, DIR_HYBRID = 3;

    private Bfsx() {
    }

    // ---- context: replaces new JavaSparkContext(...) + addJar (BfsSpark.java:50-51), spark.stop (:120) ----
    public static native long init(int device) throws IOException;

    /**
     * A group context of nranks ranks in this process (bfsx_init_group): graphs loaded on it are 1-D partitioned
     * over the ranks (one per GPU; ranks share a GPU when fewer are visible) and every call below on such a graph
     * runs all ranks and returns once -- the Spark workers of the reference's cluster (BfsSpark.java:44,50).
     */
    public static native long initGroup(int nranks) throws IOException;

    /** Ranks of a context (1 for init). */
    public static native int groupSize(long ctx);

    public static native void setOption(long ctx, String key, String value);

    public static native void finalizeContext(long ctx);

    // ---- graph: replaces GraphFileUtil.convert (BfsSpark.java:55, GraphFileUtil.java:45-69) ---------------
    public static native long loadAlgs4(long ctx, String path) throws IOException;

    public static native long fromEdges(long ctx, long nv, int[] u, int[] v);

    public static native long nv(long graph);

    public static native long nnz(long graph);

    /** CSR of the neighbour sets: rowOff (nv+1 longs) and col (nnz ints), either may be null. */
    public static native void csr(long graph, ByteBuffer rowOff, ByteBuffer col);

    public static native void free(long graph);

    // ---- the level loop: replaces BfsSpark.java:57-118 --------------------------------------------------
    /**
     * Breadth-first search from {@code source}.  dist: nv ints (Integer.MAX_VALUE = unreached, the
     * reference's WHITE distance), parent: nv longs (-1 = none) or null.
     *
     * @return the number of map/reduce passes the reference runs for the same graph and source
     */
    public static native int bfs(long graph, long source, ByteBuffer dist, ByteBuffer parent) throws IOException;

    /** Cumulative device time of every pass (the Stopwatch behind "Elapsed time [k]", BfsSpark.java:112). */
    public static native double[] levelTimesMs(long graph);

    /** Graph500 validation of the last result on the device: violating vertices (0 = exact BFS distances). */
    public static native long validate(long graph);

    // ---- multi-GPU: one JVM (executor) per GPU, replaces the reduceByKey shuffle (BfsSpark.java:90) -------
    /** 128 bytes: rank 0 creates them, a Spark Broadcast<byte[]> (or any channel) ships them. */
    public static native byte[] commUniqueId();

    /**
     * Device time (ms[4]) and calls (calls[4]) per collective kind of the last distributed BFS on this rank, with
     * option "comm_timing" on: level-close all-reduces, pair-count all-to-alls, pair / id all-to-allvs, frontier
     * all-gathers (bfsx_comm_times).  Take the max over ranks.
     */
    public static native void commTimes(long graph, double[] ms, long[] calls) throws IOException;

    public static native void commInit(long ctx, int rank, int nranks, byte[] id);

    public static native long distKronecker(long ctx, int scale, int edgefactor, long seed, int rank, int nranks);

    public static native long distFromEdges(long ctx, long nv, int[] u, int[] v, int rank, int nranks);

    /** Collective: every rank passes the same source; returns the number of passes. */
    public static native int distBfs(long graph, long source);

    /** This rank's rows [vLo, vLo + nv) of the last result (dist ints, parent longs or null). */
    public static native void result(long graph, ByteBuffer dist, ByteBuffer parent);

    /** {nvGlobal, vLo, nvLocal, chunk, rank, nranks} */
    public static native long[] partition(long graph);

    // ---- helpers -------------------------------------------------------------------------------------
    public static ByteBuffer ints(long n) {
        return ByteBuffer.allocateDirect(checkedInt(n * 4)).order(ByteOrder.nativeOrder());
    }

    public static ByteBuffer longs(long n) {
        return ByteBuffer.allocateDirect(checkedInt(n * 8)).order(ByteOrder.nativeOrder());
    }

    /** long -> int, failing on overflow (Java 7: Math.toIntExact is Java 8, the reference targets 1.7, pom.xml:16). */
    public static int checkedInt(long x) {
        if (x < Integer.MIN_VALUE || x > Integer.MAX_VALUE)
            throw new ArithmeticException("integer overflow: " + x);
        return (int) x;
    }
}
