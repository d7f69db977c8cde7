// bfsx_spark.cpp -- C++ host twin of the reference's entry point BfsSpark.main
// (src/main/java/it/unitn/bd/bfs/BfsSpark.java:43-121), driving libbfsx.so through the C-ABI.
//
// No JDK exists in this image, so the Java host cannot be compiled here; this twin keeps the same
// inputs and outputs so a user of the reference can switch without changing files:
//   - configuration: service.properties read from the working directory with the reference's keys
//     (ServiceConfiguration.java:30-43): app-name, ip, port, jar, problemFiles (comma-separated,
//     Splitter.on(",") -- no trimming).  Optional keys added here, defaults = reference behaviour:
//       source=0 (GraphFileUtil.java:28)  device=0  direction=auto|topdown|bottomup
//       devices=1 (N > 1: one call runs N ranks of a 1-D vertex partition inside this process, bfsx_init_group --
//         an RCCL clique over N GPUs, or an in-process group when fewer GPUs are visible; the Spark workers of
//         the reference's cluster, BfsSpark.java:44,50)
//       writeInitial=true (problemFile_0, GraphFileUtil.java:68)  writePaths=true
//       dumpLevels=false (every intermediate problemFile_<k>, BfsSpark.java:115-116)
//       validate=false (Graph500-style check of the result on the device, bfsx_validate; logged)
//   - input: algs4 edge lists, parsed with GraphFileUtil.convert semantics (inside libbfsx.so)
//   - output: problemFile_<k> in Vertex.toString format  id|[n, ...]|[path]|distance|COLOR
//     (Vertex.java:123-125), one line per vertex, k = number of map/reduce passes; the final file has
//     no GRAY vertex, exactly like the reference's last file (BfsSpark.java:117)
//   - log lines: "Application name", "Problem file", "Elapsed time [k] ==> <Stopwatch>" with Guava 18
//     Stopwatch.toString: String.format("%.4g %s") of the integer nanoseconds in the chosen unit, Java
//     %g rules (4 significant digits, trailing zeros kept, HALF_UP on the shortest decimal form)
//     (BfsSpark.java:45-48,54,112)
//   - neighbour lists in java.util.HashSet iteration order (Vertex.java:124 prints the set): the set is
//     filled by add() in file order (GraphFileUtil.java:64-65) and re-filled in its own iteration order
//     on every pass (Vertex.java:54-57), so every file lists a row by bucket index
//     (h ^ h >>> 16) & (table - 1), insertion order inside a bucket, table = the smallest power of two
//     >= 16 holding the row at load factor 0.75 (Java 8 HashMap).  Unpinned: the JVM the reference ran
//     on (pom.xml targets 1.7; a Java 7 HashMap hashes and orders buckets differently) and bins of >= 8
//     colliding ids in a table >= 64 (Java 8 treeifies those); the ORDER OF THE LINES of problemFile_k,
//     k >= 1, is Spark's collectAsMap order (BfsSpark.java:110) and is written here in id order.
// Deliberate difference: files are written with truncation (the reference opens with CREATE only and
// leaves stale tails behind a shorter rewrite, BfsSpark.java:27,116).
#include <algorithm>
#include <charconv>
#include <chrono>
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <sys/time.h>
#include <vector>

#include "bfsx.h"

namespace {

// ---- logging in the reference's log4j2 pattern (log4j2.xml:5) --------------------------------------
void log_line(const char *level, const char *method, int line, const std::string &msg) {
    struct timeval tv;
    gettimeofday(&tv, nullptr);
    struct tm tmv;
    localtime_r(&tv.tv_sec, &tmv);
    std::printf("%02d:%02d:%02d.%03d %-5s it.unitn.bd.bfs.BfsSpark:%s(BfsSpark.java:%d) - %s\n", tmv.tm_hour,
                tmv.tm_min, tmv.tm_sec, (int)(tv.tv_usec / 1000), level, method, line, msg.c_str());
    std::fflush(stdout);
}

// Java's String.format("%.4g", v) for v >= 0 (java.util.Formatter GENERAL conversion): the shortest
// decimal form of v (Double.toString's digits) rounded HALF_UP to 4 significant digits; plain notation
// when the rounded value is in [1e-4, 1e4), else d.ddde+XX; trailing zeros kept (1.5 -> "1.500").
std::string java_format_4g(double v) {
    if (!(v > 0.0)) return "0.000";
    char buf[64];
    const auto r = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::scientific); // shortest
    const std::string sci(buf, r.ptr);
    const size_t epos = sci.find('e');
    std::string dig;
    for (size_t i = 0; i < epos; i++)
        if (sci[i] != '.') dig += sci[i];
    int exp10 = std::atoi(sci.c_str() + epos + 1); // v = d.ddd * 10^exp10
    if (dig.size() > 4) {
        const bool up = dig[4] >= '5';
        dig.resize(4);
        if (up) {
            int i = 3;
            while (i >= 0 && dig[i] == '9') dig[i--] = '0';
            if (i >= 0) {
                dig[i]++;
            } else { // 9999.5 -> 1000e+1
                dig = "1000";
                exp10++;
            }
        }
    }
    while (dig.size() < 4) dig += '0';
    std::string out;
    if (exp10 >= -4 && exp10 < 4) {
        if (exp10 >= 0) {
            out = dig.substr(0, exp10 + 1);
            if (exp10 < 3) out += "." + dig.substr(exp10 + 1);
        } else {
            out = "0." + std::string(-exp10 - 1, '0') + dig;
        }
    } else {
        char e[16];
        std::snprintf(e, sizeof(e), "e%c%02d", exp10 < 0 ? '-' : '+', exp10 < 0 ? -exp10 : exp10);
        out = dig.substr(0, 1) + "." + dig.substr(1) + e;
    }
    return out;
}

// Guava 18 Stopwatch.toString (Stopwatch.java: chooseUnit + String.format("%.4g %s")): the elapsed
// integer nanoseconds in the largest unit they reach (d, h, min, s, ms, μs, ns).
std::string stopwatch_string(int64_t nanos) {
    static const struct {
        int64_t scale;
        const char *abbr;
    } units[] = {{86400000000000LL, "d"}, {3600000000000LL, "h"}, {60000000000LL, "min"}, {1000000000LL, "s"},
                 {1000000LL, "ms"},       {1000LL, "μs"},       {1LL, "ns"}};
    for (const auto &u : units)
        if (nanos / u.scale > 0 || u.scale == 1)
            return java_format_4g((double)nanos / (double)u.scale) + " " + u.abbr;
    return "0.000 ns";
}

// ---- java.util.Properties (subset: comments, '=' / ':' / whitespace separators, continuation lines,
// backslash escapes) --------------------------------------------------------------------------------
bool load_properties(const std::string &path, std::map<std::string, std::string> &out) {
    std::ifstream in(path);
    if (!in) return false;
    std::string raw, logical;
    std::vector<std::string> lines;
    while (std::getline(in, raw)) {
        if (!raw.empty() && raw.back() == '\r') raw.pop_back();
        size_t s = raw.find_first_not_of(" \t\f");
        std::string t = (s == std::string::npos) ? "" : raw.substr(s);
        if (logical.empty() && (t.empty() || t[0] == '#' || t[0] == '!')) continue;
        // count trailing backslashes: odd -> continuation
        size_t nb = 0;
        while (nb < t.size() && t[t.size() - 1 - nb] == '\\') nb++;
        if (nb % 2 == 1) {
            logical += t.substr(0, t.size() - 1);
            continue;
        }
        logical += t;
        lines.push_back(logical);
        logical.clear();
    }
    if (!logical.empty()) lines.push_back(logical);
    auto unescape = [](const std::string &x) {
        std::string r;
        for (size_t i = 0; i < x.size(); i++) {
            if (x[i] == '\\' && i + 1 < x.size()) {
                char c = x[++i];
                r += c == 't' ? '\t' : c == 'n' ? '\n' : c == 'r' ? '\r' : c == 'f' ? '\f' : c;
            } else {
                r += x[i];
            }
        }
        return r;
    };
    for (const auto &l : lines) {
        size_t i = 0;
        std::string key;
        while (i < l.size() && l[i] != '=' && l[i] != ':' && l[i] != ' ' && l[i] != '\t' && l[i] != '\f') {
            if (l[i] == '\\' && i + 1 < l.size()) {
                key += l[i];
                i++;
            }
            key += l[i++];
        }
        while (i < l.size() && (l[i] == ' ' || l[i] == '\t' || l[i] == '\f')) i++;
        if (i < l.size() && (l[i] == '=' || l[i] == ':')) i++;
        while (i < l.size() && (l[i] == ' ' || l[i] == '\t' || l[i] == '\f')) i++;
        out[unescape(key)] = unescape(l.substr(i));
    }
    return true;
}

std::vector<std::string> split_commas(const std::string &s) { // Splitter.on(",").splitToList
    std::vector<std::string> r;
    size_t a = 0;
    while (true) {
        size_t b = s.find(',', a);
        r.push_back(s.substr(a, b == std::string::npos ? std::string::npos : b - a));
        if (b == std::string::npos) break;
        a = b + 1;
    }
    return r;
}

bool truthy(const std::string &v) { return v == "true" || v == "TRUE" || v == "True" || v == "1"; }

// ---- neighbour rows in java.util.HashSet iteration order (see the header) ----------------------------
// Rows are filled in file order (GraphFileUtil.java:64-65: vertex1 gets vertex2, then vertex2 gets
// vertex1; a repeated neighbour or a self-loop's second add changes nothing), then each row is stably
// ordered by its Java 8 HashMap bucket.  Out: off/col of the rows in output order.
int hashset_rows(const std::string &file, int64_t nv, std::vector<int64_t> &off, std::vector<uint32_t> &col) {
    int64_t pnv = 0, m = 0;
    uint32_t *u = nullptr, *v = nullptr;
    if (int rc = bfsx_parse_algs4(file.c_str(), &pnv, &m, &u, &v)) return rc;
    if (pnv != nv) {
        bfsx_free_host(u);
        bfsx_free_host(v);
        return BFSX_E_PARSE;
    }
    std::vector<int64_t> cnt(nv + 1, 0);
    for (int64_t i = 0; i < m; i++) {
        cnt[u[i] + 1]++;
        cnt[v[i] + 1]++;
    }
    for (int64_t x = 0; x < nv; x++) cnt[x + 1] += cnt[x];
    std::vector<uint32_t> raw(cnt[nv]);
    std::vector<int64_t> cur(cnt.begin(), cnt.end() - 1);
    for (int64_t i = 0; i < m; i++) { // insertion order of every row
        raw[cur[u[i]]++] = v[i];
        raw[cur[v[i]]++] = u[i];
    }
    bfsx_free_host(u);
    bfsx_free_host(v);
    off.assign(nv + 1, 0);
    col.clear();
    col.reserve(raw.size());
    std::vector<uint32_t> row;
    std::vector<std::pair<uint32_t, uint32_t>> keyed; // (bucket, insertion rank)
    for (int64_t x = 0; x < nv; x++) {
        row.assign(raw.begin() + cnt[x], raw.begin() + cnt[x + 1]);
        // first occurrences, in order
        std::vector<std::pair<uint32_t, uint32_t>> firsts;
        firsts.reserve(row.size());
        for (uint32_t i = 0; i < row.size(); i++) firsts.push_back({row[i], i});
        std::stable_sort(firsts.begin(), firsts.end(),
                         [](const std::pair<uint32_t, uint32_t> &a, const std::pair<uint32_t, uint32_t> &b) {
                             return a.first < b.first;
                         });
        std::vector<std::pair<uint32_t, uint32_t>> uniq; // (insertion rank, id)
        for (size_t i = 0; i < firsts.size(); i++)
            if (i == 0 || firsts[i].first != firsts[i - 1].first) uniq.push_back({firsts[i].second, firsts[i].first});
        std::sort(uniq.begin(), uniq.end());
        uint64_t table = 16;
        while (uniq.size() > table * 3 / 4) table *= 2; // resize when size > 0.75 * capacity
        keyed.clear();
        for (uint32_t i = 0; i < uniq.size(); i++) {
            const uint32_t h = uniq[i].second;
            keyed.push_back({(uint32_t)((h ^ (h >> 16)) & (table - 1)), i});
        }
        std::stable_sort(keyed.begin(), keyed.end()); // ties: insertion rank ascending
        for (const auto &k : keyed) col.push_back(uniq[k.second].second);
        off[x + 1] = (int64_t)col.size();
    }
    return BFSX_OK;
}

// ---- Vertex.toString writer (Vertex.java:123-125) -------------------------------------------------
// state after map/reduce pass `k` (k = levels: final state).  A vertex at distance d < k is BLACK,
// d == k is GRAY (discovered by pass k), d > k or unreachable is WHITE with Integer.MAX_VALUE and the
// initial path [source] (GraphFileUtil.java:54-56).
bool write_state(const std::string &file, int64_t nv, const std::vector<int64_t> &off,
                 const std::vector<uint32_t> &col, const std::vector<int32_t> &dist,
                 const std::vector<int64_t> &parent, int64_t source, int64_t k, bool paths) {
    FILE *f = std::fopen(file.c_str(), "wb");
    if (!f) return false;
    std::vector<uint32_t> row, path;
    std::string buf;
    buf.reserve(1 << 20);
    for (int64_t v = 0; v < nv; v++) {
        row.assign(col.begin() + off[v], col.begin() + off[v + 1]); // already in HashSet order
        const int32_t d = dist[v];
        const bool reached = d != INT32_MAX && d <= k;
        buf += std::to_string(v);
        buf += "|[";
        for (size_t i = 0; i < row.size(); i++) {
            if (i) buf += ", ";
            buf += std::to_string(row[i]);
        }
        buf += "]|[";
        if (reached && paths) {
            path.clear();
            for (int64_t x = v; x != source; x = parent[x]) path.push_back((uint32_t)x);
            path.push_back((uint32_t)source);
            for (size_t i = path.size(); i-- > 0;) {
                buf += std::to_string(path[i]);
                if (i) buf += ", ";
            }
        } else {
            buf += std::to_string(source);
        }
        buf += "]|";
        buf += std::to_string(reached ? d : INT32_MAX);
        buf += "|";
        buf += !reached ? "WHITE" : (d == k && k > 0) ? "GRAY" : (k == 0 ? "GRAY" : "BLACK");
        if (v + 1 < nv) buf += "\n"; // NEW_LINE.join (BfsSpark.java:115): no trailing newline
        if (buf.size() > (1 << 20)) {
            std::fwrite(buf.data(), 1, buf.size(), f);
            buf.clear();
        }
    }
    std::fwrite(buf.data(), 1, buf.size(), f);
    return std::fclose(f) == 0;
}

int run_problem(bfsx_ctx *ctx, const std::string &problem, int64_t source, bool write_initial, bool paths,
                bool dump_levels, bool validate) {
    log_line("INFO", "main", 54, "Problem file: " + problem);
    bfsx_graph *g = nullptr;
    int rc = bfsx_graph_load_algs4(ctx, problem.c_str(), &g); // GraphFileUtil.convert (BfsSpark.java:55)
    if (rc) {
        log_line("ERROR", "main", 55, std::string("GraphFileUtil.convert failed: ") + bfsx_last_error());
        return rc;
    }
    const int64_t nv = bfsx_graph_nv(g), nnz = bfsx_graph_nnz(g);
    std::vector<int64_t> off(nv + 1);
    std::vector<uint32_t> col(std::max<int64_t>(nnz, 1));
    std::vector<int32_t> dist(nv, INT32_MAX);
    std::vector<int64_t> parent(nv, -1);
    // the rows as the reference prints them (the device CSR holds the same sets, degree-ordered)
    if ((rc = hashset_rows(problem, nv, off, col))) goto out;
    if ((int64_t)col.size() != nnz) {
        log_line("ERROR", "main", 55, "adjacency of the written rows differs from the device graph");
        rc = BFSX_E_PARSE;
        goto out;
    }
    if (source < 0 || source >= nv) {
        log_line("ERROR", "main", 55, "source vertex outside the graph");
        rc = BFSX_E_RANGE;
        goto out;
    }
    if (write_initial) {
        dist[source] = 0;
        parent[source] = source;
        if (!write_state(problem + "_0", nv, off, col, dist, parent, source, 0, paths)) {
            rc = BFSX_E_IO;
            goto out;
        }
    }
    {
        bfsx_stats st{};
        if ((rc = bfsx_bfs(g, source, dist.data(), parent.data(), &st))) {
            log_line("ERROR", "main", 61, std::string("bfs failed: ") + bfsx_last_error());
            goto out;
        }
        std::vector<double> cum(st.levels);
        bfsx_level_times(g, cum.data(), st.levels);
        for (int k = 1; k <= st.levels; k++) {
            log_line("INFO", "main", 112, "Elapsed time [" + std::to_string(k) + "] ==> " +
                                              stopwatch_string(std::llround(cum[k - 1] * 1e6)));
            const bool last = k == st.levels;
            if ((dump_levels || last) &&
                !write_state(problem + "_" + std::to_string(k), nv, off, col, dist, parent, source, k, paths)) {
                log_line("ERROR", "main", 116, "cannot write " + problem + "_" + std::to_string(k));
                rc = BFSX_E_IO;
                goto out;
            }
        }
        char msg[256];
        std::snprintf(msg, sizeof(msg),
                      "BFS done: %d passes (%d top-down, %d bottom-up), %" PRId64 " reached, %" PRId64
                      " input edges in component, %.3f ms device, %.3f GTEPS",
                      st.levels, st.topdown_levels, st.bottomup_levels, st.reached, st.m_comp, st.t_bfs_ms,
                      st.t_bfs_ms > 0 ? st.m_comp / (st.t_bfs_ms * 1e6) : 0.0);
        log_line("INFO", "main", 117, msg);
        if (validate) {
            int64_t bad = 0, first = -1;
            if ((rc = bfsx_validate(g, source, &bad, &first, nullptr, nullptr))) {
                log_line("ERROR", "main", 117, std::string("validation failed to run: ") + bfsx_last_error());
                goto out;
            }
            log_line(bad ? "ERROR" : "INFO", "main", 117,
                     bad ? "Validation: " + std::to_string(bad) + " violating vertices, first " + std::to_string(first)
                         : std::string("Validation: OK (Graph500 rules, exact BFS distances)"));
            if (bad) rc = BFSX_E_ARG;
        }
    }
out:
    bfsx_graph_free(g);
    return rc;
}

} // namespace

int main(int argc, char **argv) {
    std::string props_path = "service.properties"; // ServiceConfiguration.CONFIGURATION_FILE (:18)
    for (int i = 1; i < argc; i++) {
        if (!std::strcmp(argv[i], "--properties") && i + 1 < argc) props_path = argv[++i];
        else if (!std::strcmp(argv[i], "--format-nanos")) { // the Stopwatch format of each argument (tests)
            for (int j = i + 1; j < argc; j++) std::printf("%s\n", stopwatch_string(std::strtoll(argv[j], nullptr, 10)).c_str());
            return 0;
        } else if (!std::strcmp(argv[i], "--help")) {
            std::printf("usage: bfsx_spark [--properties service.properties] | --format-nanos N...\n");
            return 0;
        }
    }
    std::map<std::string, std::string> p;
    if (!load_properties(props_path, p) || !p.count("problemFiles")) {
        // the reference logs and swallows this (ServiceConfiguration.java:40-42), then fails on the
        // null problem-file list in main
        std::fprintf(stderr, "Failed to load service configuration! (%s)\n", props_path.c_str());
        return 2;
    }
    auto get = [&](const char *k, const char *def) { return p.count(k) ? p[k] : std::string(def); };
    const std::string master = "spark://" + get("ip", "") + ":" + get("port", "");
    log_line("INFO", "main", 45, "Application name: " + get("app-name", ""));
    const std::vector<std::string> files = split_commas(p["problemFiles"]);
    {
        std::string lst = "[";
        for (size_t i = 0; i < files.size(); i++) lst += (i ? ", " : "") + files[i];
        log_line("INFO", "main", 46, "Problem files path: " + lst + "]");
    }
    log_line("INFO", "main", 47, "Using JAR file: " + get("jar", ""));
    const int devices = std::atoi(get("devices", "1").c_str());
    if (devices < 1 || devices > 64) {
        std::fprintf(stderr, "devices must be in [1, 64]\n");
        return 2;
    }
    bfsx_ctx *ctx = nullptr;
    int rc = BFSX_OK;
    if (devices == 1) {
        log_line("INFO", "main", 48, "Connecting to: " + master + " (replaced by libbfsx on HIP device " +
                                         get("device", "0") + ")");
        rc = bfsx_init(std::atoi(get("device", "0").c_str()), &ctx);
    } else {
        log_line("INFO", "main", 48, "Connecting to: " + master + " (replaced by libbfsx: " + std::to_string(devices) +
                                         " ranks of a 1-D vertex partition, one per HIP device)");
        rc = bfsx_init_group(devices, &ctx);
    }
    if (rc) {
        std::fprintf(stderr, "bfsx_init failed: %s\n", bfsx_last_error());
        return 3;
    }
    if ((rc = bfsx_set_option(ctx, "direction", get("direction", "auto").c_str()))) {
        std::fprintf(stderr, "%s\n", bfsx_last_error());
        bfsx_finalize(ctx);
        return 2;
    }
    const int64_t source = std::strtoll(get("source", "0").c_str(), nullptr, 10);
    const bool write_initial = truthy(get("writeInitial", "true"));
    const bool paths = truthy(get("writePaths", "true"));
    const bool dump = truthy(get("dumpLevels", "false"));
    const bool validate = truthy(get("validate", "false"));
    int status = 0;
    for (const auto &f : files) { // BfsSpark.java:53
        rc = run_problem(ctx, f, source, write_initial, paths, dump, validate);
        if (rc) {
            status = rc == BFSX_E_IO ? 4 : 5;
            break; // an exception escapes main in the reference (BfsSpark.java:43 throws Exception)
        }
    }
    bfsx_finalize(ctx);
    return status;
}
