package it.unitn.bd.bfs;

import it.unitn.bd.ServiceConfiguration;
import it.unitn.bd.bfs.graph.Color;
import it.unitn.bd.bfs.graph.Vertex;
import org.apache.logging.log4j.LogManager;
import org.apache.logging.log4j.Logger;

import java.io.BufferedReader;
import java.io.FileInputStream;
import java.io.IOException;
import java.io.InputStream;
import java.io.InputStreamReader;
import java.nio.ByteBuffer;
import java.nio.file.Files;
import java.nio.file.Paths;
import java.nio.file.StandardOpenOption;
import java.util.ArrayList;
import java.util.HashSet;
import java.util.LinkedList;
import java.util.List;
import java.util.Properties;
import java.util.Set;

/**
 * The reference's entry point with its per-problem-file block (BfsSpark.java:53-119) on the MI355X:
 * GraphFileUtil.convert and the map/reduceByKey level loop are replaced by two calls into libbfsx.so
 * (Bfsx.loadAlgs4 + Bfsx.bfs); configuration (service.properties through ServiceConfiguration), the
 * log lines and the files problemFile_0 / problemFile_passes keep the reference's format, written with
 * the reference's own Vertex.toString.
 *
 * Added to the reference's source tree next to BfsSpark (it uses ServiceConfiguration, Vertex and
 * Color from there) with Bfsx.java, and run as
 *   java -Djava.library.path=<dir of libbfsx_jni.so and libbfsx.so> -cp <jar> it.unitn.bd.bfs.BfsGpu
 * Options, each read from a system property (-Dbfsx.<key>) or else from the same service.properties key (the
 * reference's keys are read by its ServiceConfiguration, ServiceConfiguration.java:35-39; these are added, with
 * defaults that keep the reference's behaviour, SURVEY.md 5):
 *   device (HIP ordinal, default 0);  devices (default 1; N > 1: N ranks of a 1-D vertex partition in this
 *   process, Bfsx.initGroup -- one GPU each, or sharing the visible ones);  direction (auto|topdown|bottomup);
 *   dumpLevels (true: every pass's problemFile_k, as the reference writes them, BfsSpark.java:115-116; default
 *   false: problemFile_0 and the last pass only);  validate (true: Graph500 validation of every result on the
 *   device, logged).
 *
 * Differences kept from the C++ twin (bfs-with-mapreduce_amd/host/bfsx_spark.cpp): the final file lists
 * vertices in id order (the reference's order is Spark's collectAsMap order, BfsSpark.java:110), and
 * files are truncated when rewritten (the reference opens with CREATE only, BfsSpark.java:116).
 * Not compiled in this repository's image (it has no JDK): build with java/Makefile.
 */
public final class BfsGpu {

    private static final Logger logger = LogManager.getLogger();

    private static final int SOURCE_VERTEX = 0; // GraphFileUtil.java:28

    private static final Properties SERVICE = new Properties();

    static {
        // the same file ServiceConfiguration reads (ServiceConfiguration.java:18,30-33), for the added keys
        try (InputStream in = new FileInputStream("service.properties")) {
            SERVICE.load(in);
        } catch (IOException e) {
            logger.warn("service.properties not readable for the bfsx keys: " + e.getMessage());
        }
    }

    private BfsGpu() {
    }

    /** -Dbfsx.key, else the service.properties key, else the default. */
    static String option(String key, String def) {
        final String p = System.getProperty("bfsx." + key);
        return p != null ? p : SERVICE.getProperty(key, def);
    }

    public static void main(String[] args) throws Exception {
        logger.info("Application name: " + ServiceConfiguration.getAppName());
        logger.info("Problem files path: " + ServiceConfiguration.getProblemFiles());
        final int devices = Integer.parseInt(option("devices", "1"));
        final long ctx;
        if (devices > 1) {
            logger.info("Connecting to: " + devices + " ranks of a 1-D vertex partition, one per HIP device (libbfsx)");
            ctx = Bfsx.initGroup(devices);
        } else {
            final int device = Integer.parseInt(option("device", "0"));
            logger.info("Connecting to: HIP device " + device + " (libbfsx)");
            ctx = Bfsx.init(device);
        }
        try {
            Bfsx.setOption(ctx, "direction", option("direction", "auto"));
            for (String problemFile : ServiceConfiguration.getProblemFiles()) {
                logger.info("Problem file: " + problemFile);
                run(ctx, problemFile);
            }
        } finally {
            Bfsx.finalizeContext(ctx);
        }
    }

    private static void run(long ctx, String problemFile) throws IOException {
        final long g = Bfsx.loadAlgs4(ctx, problemFile); // GraphFileUtil.convert (BfsSpark.java:55)
        try {
            final int nv = Bfsx.checkedInt(Bfsx.nv(g));
            final List<Set<Integer>> neighbours = neighbourSets(problemFile, nv);
            final ByteBuffer dist = Bfsx.ints(nv), parent = Bfsx.longs(nv);
            write(problemFile + "_0", neighbours, null, null, 0); // the initial state (GraphFileUtil.java:68)
            final int passes = Bfsx.bfs(g, SOURCE_VERTEX, dist, parent); // BfsSpark.java:57-118
            final double[] cum = Bfsx.levelTimesMs(g);
            final boolean dumpLevels = Boolean.parseBoolean(option("dumpLevels", "false"));
            for (int k = 1; k <= passes; k++) {
                logger.info("Elapsed time [" + k + "] ==> " + stopwatch(Math.round(cum[k - 1] * 1e6)));
                // the state after pass k, as the reference writes it every pass (BfsSpark.java:115-116)
                if (dumpLevels || k == passes) write(problemFile + "_" + k, neighbours, dist, parent, k);
            }
            if (Boolean.parseBoolean(option("validate", "false"))) {
                final long bad = Bfsx.validate(g);
                logger.info(bad == 0 ? "Validation: OK (Graph500 rules, exact BFS distances)"
                                     : "Validation: " + bad + " violating vertices");
            }
        } finally {
            Bfsx.free(g);
        }
    }

    /**
     * The neighbour sets as the reference holds them: a HashSet per vertex filled by add() in file order
     * (GraphFileUtil.java:60-66), so Vertex.toString prints them in the same iteration order.  The device
     * graph holds the same sets; this pass exists only to print them.
     */
    private static List<Set<Integer>> neighbourSets(String problemFile, int nv) throws IOException {
        final List<Set<Integer>> sets = new ArrayList<>(nv);
        for (int i = 0; i < nv; i++) sets.add(new HashSet<Integer>());
        try (BufferedReader reader = new BufferedReader(new InputStreamReader(new FileInputStream(problemFile)))) {
            reader.readLine(); // vertex count (already parsed by the library)
            reader.readLine(); // edge count, unused
            String line;
            while ((line = reader.readLine()) != null) {
                final int sp = line.indexOf(' ');
                final int sp2 = line.indexOf(' ', sp + 1);
                final int a = Integer.parseInt(line.substring(0, sp));
                final int b = Integer.parseInt(sp2 < 0 ? line.substring(sp + 1) : line.substring(sp + 1, sp2));
                sets.get(a).add(b);
                sets.get(b).add(a);
            }
        }
        return sets;
    }

    /**
     * The state after pass `pass` (the map/reduce semantics of BfsSpark.java:66-108): pass 0 is the source GRAY,
     * everything else WHITE; after pass k a vertex at distance d < k is BLACK, d == k GRAY (discovered by that
     * pass), and d > k or unreachable WHITE with Integer.MAX_VALUE and the initial path [source].
     */
    private static void write(String file, List<Set<Integer>> neighbours, ByteBuffer dist, ByteBuffer parent, int pass)
            throws IOException {
        final StringBuilder out = new StringBuilder();
        final LinkedList<Integer> start = new LinkedList<>();
        start.add(SOURCE_VERTEX);
        for (int v = 0; v < neighbours.size(); v++) {
            final Vertex vertex;
            if (pass == 0) {
                vertex = v == SOURCE_VERTEX ? new Vertex(v, neighbours.get(v), start, 0, Color.GRAY)
                                            : new Vertex(v, neighbours.get(v), start, Integer.MAX_VALUE, Color.WHITE);
            } else {
                final int d = dist.getInt(4 * v);
                if (d == Integer.MAX_VALUE || d > pass) {
                    vertex = new Vertex(v, neighbours.get(v), start, Integer.MAX_VALUE, Color.WHITE);
                } else {
                    final LinkedList<Integer> path = new LinkedList<>();
                    for (long x = v; ; x = parent.getLong(8 * (int) x)) {
                        path.addFirst((int) x);
                        if (x == SOURCE_VERTEX) break;
                    }
                    vertex = new Vertex(v, neighbours.get(v), path, d, d == pass ? Color.GRAY : Color.BLACK);
                }
            }
            if (v > 0) out.append('\n'); // Joiner.on("\n") (BfsSpark.java:115)
            out.append(vertex);
        }
        Files.write(Paths.get(file), out.toString().getBytes(), StandardOpenOption.CREATE,
                StandardOpenOption.TRUNCATE_EXISTING, StandardOpenOption.WRITE);
    }

    /** Guava 18 Stopwatch.toString of an elapsed time in nanoseconds (BfsSpark.java:112). */
    static String stopwatch(long nanos) {
        final long[] scale = {86_400_000_000_000L, 3_600_000_000_000L, 60_000_000_000L, 1_000_000_000L, 1_000_000L,
                1_000L, 1L};
        final String[] abbr = {"d", "h", "min", "s", "ms", "μs", "ns"};
        int u = 0;
        while (u < scale.length - 1 && nanos / scale[u] == 0) u++;
        return String.format("%.4g %s", (double) nanos / scale[u], abbr[u]);
    }
}
