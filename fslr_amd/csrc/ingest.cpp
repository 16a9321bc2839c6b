// ingest.cpp — threaded reader for `{name}.mappings.bed` (include/fslr_ingest.h).
// Host-only C++17; built with g++ into fslr_amd/libfslr_ingest.so.
//
// Layout: the file is mapped read-only (threads fault its pages in parallel); line starts are found by a
// per-thread newline count + prefix sum; a column is produced by re-walking each
// line to its k-th tab (the file stays hot in the CPU caches per chunk, and only
// the requested columns are ever materialised).
#include "fslr_ingest.h"

#include <algorithm>
#include <memory>
#include <cctype>
#include <emmintrin.h>
#include <charconv>
#include <cmath>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include <cerrno>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

// A vector allocator that leaves new int64 elements uninitialised (the line index is filled by
// threads; zero-filling 1+ GB first on one thread costs more than the scan).
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U> struct rebind { using other = NoInitAlloc<U>; };
    NoInitAlloc() = default;
    template <class U> NoInitAlloc(const NoInitAlloc<U> &) {}
    template <class U> void construct(U *p) noexcept { ::new (static_cast<void *>(p)) U; }
    template <class U, class... A> void construct(U *p, A &&...a) { ::new (static_cast<void *>(p)) U(std::forward<A>(a)...); }
};

struct FslrTsv {
    const char *data = nullptr;           // the mapped file (size bytes)
    size_t size = 0;
    void *map = nullptr;                  // mmap base (nullptr for an empty file)
    ~FslrTsv() { if (map) munmap(map, size); }
    std::vector<int64_t, NoInitAlloc<int64_t>> line;   // [rows starts | file size | rows ends] (header excluded)
    std::vector<std::string> names;       // header
    int n_threads = 1;
    // last factorize result per column
    std::vector<std::vector<std::string_view>> uniq;
};

namespace {

void set_err(char *err, size_t n, const std::string &m) {
    if (err && n) { std::snprintf(err, n, "%s", m.c_str()); }
}

template <class F>
void parallel_for(int64_t n, int threads, F f) {
    if (n <= 0) return;
    int t = (int)std::min<int64_t>(threads, std::max<int64_t>(1, n / 4096));
    if (t <= 1) { f(0, n, 0); return; }
    std::vector<std::thread> pool;
    for (int i = 0; i < t; ++i) {
        int64_t a = n * i / t, b = n * (i + 1) / t;
        pool.emplace_back([=, &f] { f(a, b, i); });
    }
    for (auto &th : pool) th.join();
}

// Field `col` of the line starting at `s` (line ends at `e`, '\n' and '\r' excluded).
inline std::string_view field(const char *s, const char *e, int col) {
    const char *p = s;
    for (int k = 0; k < col; ++k) {
        const void *q = std::memchr(p, '\t', (size_t)(e - p));
        if (!q) return std::string_view(nullptr, 0);   // missing field: pandas gives NaN
        p = (const char *)q + 1;
    }
    const void *q = std::memchr(p, '\t', (size_t)(e - p));
    const char *fe = q ? (const char *)q : e;
    return std::string_view(p, (size_t)(fe - p));
}

// Canonical decimal int64: "0" or -?[1-9][0-9]*, no "-0", in range.
inline bool canon_int(std::string_view f, int64_t *v) {
    size_t n = f.size(), i = 0;
    if (n == 0 || !f.data()) return false;
    bool neg = f[0] == '-';
    if (neg) { if (n == 1) return false; i = 1; }
    if (f[i] == '0') { if (n != i + 1 || neg) return false; *v = 0; return true; }
    if (n - i > 19) return false;
    unsigned long long x = 0;
    for (; i < n; ++i) {
        unsigned d = (unsigned char)f[i] - '0';
        if (d > 9) return false;
        x = x * 10 + d;
    }
    if (!neg && x > 9223372036854775807ULL) return false;
    if (neg && x > 9223372036854775808ULL) return false;
    *v = neg ? (int64_t)(0 - x) : (int64_t)x;
    return true;
}

// pandas' default na_values (read_csv keep_default_na=True).
bool is_na(std::string_view f) {
    static const std::string_view na[] = {"", "#N/A", "#N/A N/A", "#NA", "-1.#IND", "-1.#QNAN", "-NaN", "-nan",
                                          "1.#IND", "1.#QNAN", "<NA>", "N/A", "NA", "NULL", "NaN", "None",
                                          "n/a", "nan", "null"};
    if (!f.data() || f.empty()) return true;
    // every NA spelling is at most 8 bytes and starts with one of these
    if (f.size() > 8) return false;
    const char c0 = f[0];
    if (c0 != '#' && c0 != '-' && c0 != '1' && c0 != '<' && c0 != 'N' && c0 != 'n') return false;
    for (const std::string_view &s : na)
        if (f == s) return true;
    return false;
}

}  // namespace

extern "C" {

int fslr_tsv_open(const char *path, int n_threads, FslrTsv **out, char *err, size_t errlen) {
    *out = nullptr;
    const int fd = ::open(path, O_RDONLY);
    if (fd < 0) { set_err(err, errlen, std::string("cannot open ") + path); return FSLR_INGEST_ERROR; }
    struct stat sb;
    if (fstat(fd, &sb) != 0) { ::close(fd); set_err(err, errlen, std::string("cannot stat ") + path); return FSLR_INGEST_ERROR; }
    auto *t = new FslrTsv();
    t->size = (size_t)std::max<off_t>(0, sb.st_size);
    if (t->size) {
        t->map = mmap(nullptr, t->size, PROT_READ, MAP_PRIVATE, fd, 0);
        if (t->map == MAP_FAILED) {
            t->map = nullptr;
            ::close(fd);
            delete t;
            set_err(err, errlen, "mmap failed");
            return FSLR_INGEST_ERROR;
        }
        madvise(t->map, t->size, MADV_WILLNEED);
        t->data = static_cast<const char *>(t->map);
    } else {
        t->data = "";
    }
    ::close(fd);
    if (n_threads <= 0) {   // the CPU share, not the whole machine: OMP_NUM_THREADS, else min(cores, 16)
        const char *env = std::getenv("OMP_NUM_THREADS");
        n_threads = env ? std::atoi(env) : 0;
        if (n_threads <= 0) n_threads = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    }
    t->n_threads = std::min(n_threads, 256);
    const char *b = t->data;
    const int64_t n = (int64_t)t->size;
    {
        std::atomic<bool> quoted{false};
        const int Tq = (int)std::max<int64_t>(1, std::min<int64_t>(t->n_threads, n >> 20));
        std::vector<std::thread> qp;
        for (int i = 0; i < Tq; ++i)
            qp.emplace_back([&, i] {
                const int64_t a = n * i / Tq, e = n * (i + 1) / Tq;
                if (a < e && std::memchr(b + a, '"', (size_t)(e - a))) quoted = true;
            });
        for (auto &th : qp) th.join();
        if (quoted) { delete t; set_err(err, errlen, "quoted fields"); return FSLR_INGEST_DECLINE; }
    }
    // header
    const char *nl = (const char *)std::memchr(b, '\n', (size_t)n);
    int64_t h_end = nl ? (int64_t)(nl - b) : n;
    int64_t body = nl ? h_end + 1 : n;
    {
        std::string_view h(b, (size_t)h_end);
        if (!h.empty() && h.back() == '\r') h.remove_suffix(1);
        size_t p = 0;
        while (true) {
            size_t q = h.find('\t', p);
            t->names.emplace_back(h.substr(p, q == std::string_view::npos ? std::string_view::npos : q - p));
            if (q == std::string_view::npos) break;
            p = q + 1;
        }
    }
    // Lines: each chunk counts the non-blank line starts in it (newline scan), then fills its
    // slice of the index with them and with the end (one past its first newline) of each such
    // line; a chunk's last line may end in a later chunk and is completed by one memchr.  Blank
    // lines are skipped (skip_blank_lines=True).  Layout: line[0..rows) starts, line[rows] = n,
    // line[rows+1 ..] ends.
    const int T = t->n_threads;
    const int64_t len = n - body;
    auto chunk = [&](int i) { return std::make_pair(body + len * i / T, body + len * (i + 1) / T); };
    auto nonblank = [&](int64_t p) {   // p (a line start) begins a non-blank line
        return p < n && !(b[p] == '\n' || (b[p] == '\r' && (p + 1 >= n || b[p + 1] == '\n')));
    };
    // f(p) for every non-blank line start p in [a, e) and g(y) for every newline y in [a - 1, e - 1)
    auto walk = [&](int64_t a, int64_t e, auto &&f, auto &&g) {
        if (a >= e) return;
        if (a == body && nonblank(a)) f(a);
        int64_t x = a == body ? a : a - 1;   // a newline at a-1 makes a a start
        while (x < e - 1) {
            const void *q = std::memchr(b + x, '\n', (size_t)(e - 1 - x));
            if (!q) break;
            const int64_t y = (int64_t)((const char *)q - b);
            g(y);
            if (nonblank(y + 1)) f(y + 1);
            x = y + 1;
        }
    };
    std::vector<int64_t> base((size_t)T + 1, 0);
    std::vector<std::thread> pool;
    for (int i = 0; i < T; ++i)
        pool.emplace_back([&, i] {
            auto [a, e] = chunk(i);
            int64_t c = 0;
            walk(a, e, [&](int64_t) { ++c; }, [](int64_t) {});
            base[(size_t)i + 1] = c;
        });
    for (auto &th : pool) th.join();
    pool.clear();
    for (int i = 0; i < T; ++i) base[(size_t)i + 1] += base[(size_t)i];
    const int64_t rows = base[(size_t)T];
    t->line.resize((size_t)rows * 2 + 1);
    if (rows) madvise(t->line.data(), t->line.size() * sizeof(int64_t), MADV_HUGEPAGE);
    t->line[(size_t)rows] = n;
    int64_t *S = t->line.data(), *E = t->line.data() + rows + 1;
    for (int i = 0; i < T; ++i)
        pool.emplace_back([&, i] {
            auto [a, e] = chunk(i);
            int64_t k = base[(size_t)i];
            bool open = false;                       // S[k - 1] has no end yet
            walk(a, e, [&](int64_t p) { S[k++] = p; open = true; },
                 [&](int64_t y) { if (open) { E[k - 1] = y + 1; open = false; } });
            if (open) {                              // ends in a later chunk (or at the end of the file)
                const int64_t s0 = S[k - 1];
                const void *q = std::memchr(b + s0, '\n', (size_t)(n - s0));
                E[k - 1] = q ? (int64_t)((const char *)q - b) + 1 : n;
            }
        });
    for (auto &th : pool) th.join();
    t->uniq.assign(t->names.size(), {});
    *out = t;
    return FSLR_INGEST_OK;
}

void fslr_tsv_close(FslrTsv *t) { delete t; }

int64_t fslr_tsv_rows(const FslrTsv *t) { return (int64_t)(t->line.size() / 2); }

int fslr_tsv_cols(const FslrTsv *t) { return (int)t->names.size(); }

const char *fslr_tsv_colname(const FslrTsv *t, int col) {
    return (col >= 0 && col < (int)t->names.size()) ? t->names[col].c_str() : nullptr;
}

int fslr_tsv_find(const FslrTsv *t, const char *name) {
    for (size_t i = 0; i < t->names.size(); ++i)
        if (t->names[i] == name) return (int)i;
    return -1;
}

}  // extern "C"

namespace {
// 64-bit hash of a short string: 8-byte words folded with a multiply-xorshift mix.
inline uint64_t str_hash(std::string_view f) {
    const uint64_t k = 0x9E3779B97F4A7C15ull;
    uint64_t h = (uint64_t)f.size() * k;
    size_t i = 0;
    for (; i + 8 <= f.size(); i += 8) {
        uint64_t w;
        std::memcpy(&w, f.data() + i, 8);
        h = (h ^ w) * k;
        h ^= h >> 29;
    }
    if (i < f.size()) {
        uint64_t w = 0;
        std::memcpy(&w, f.data() + i, f.size() - i);
        h = (h ^ w) * k;
        h ^= h >> 29;
    }
    h *= 0xBF58476D1CE4E5B9ull;
    return h ^ (h >> 31);
}

// Open-addressing map string_view -> int32 id (linear probing, grown at half load).
struct StrTable {
    struct Slot { uint64_t h; const char *p; uint32_t n; int32_t id; };
    std::vector<Slot> s;
    size_t used = 0, mask = 0;
    StrTable() { s.assign(1024, Slot{0, nullptr, 0, -1}); mask = 1023; }
    void grow() {
        std::vector<Slot> o;
        o.swap(s);
        s.assign(o.size() * 2, Slot{0, nullptr, 0, -1});
        mask = s.size() - 1;
        for (const Slot &x : o)
            if (x.id >= 0) {
                size_t j = (size_t)(x.h >> 7) & mask;        // the low bits choose the merge shard
                while (s[j].id >= 0) j = (j + 1) & mask;
                s[j] = x;
            }
    }
    // the id of key f, inserting `fresh` when absent
    int32_t *find_or_insert(std::string_view f, uint64_t h, int32_t fresh) {
        if (2 * (used + 1) > s.size()) grow();
        size_t j = (size_t)(h >> 7) & mask;
        while (s[j].id >= 0) {
            if (s[j].h == h && s[j].n == f.size() && std::memcmp(s[j].p, f.data(), f.size()) == 0) return &s[j].id;
            j = (j + 1) & mask;
        }
        s[j] = Slot{h, f.data(), (uint32_t)f.size(), fresh};
        ++used;
        return &s[j].id;
    }
};

// First-appearance dictionary of one column over one chunk of rows (local ids in local order).
struct ChunkDict {
    StrTable m;
    std::vector<std::string_view> ord;
    std::vector<uint64_t> oh;
    std::string_view prev;
    int32_t prev_id = -1;
    bool have_prev = false, all_int = true, na = false;
    int32_t add(std::string_view f) {
        if (have_prev && f == prev) return prev_id;     // rows of one read are adjacent: no lookup
        if (is_na(f)) { na = true; return 0; }
        int64_t d;
        if (all_int && !canon_int(f, &d)) all_int = false;
        const uint64_t h = str_hash(f);
        const int32_t id = *m.find_or_insert(f, h, (int32_t)ord.size());
        if (id == (int32_t)ord.size()) { ord.push_back(f); oh.push_back(h); }
        prev = f;
        prev_id = id;
        have_prev = true;
        return id;
    }
};

// The chunks' dictionaries (chunk c = rows [rows c / T, rows (c+1) / T), codes holding local ids)
// merged into pd.factorize codes: sharded by hash, shard s walks the chunks in order, so the first
// chunk holding a key is its global first appearance; global ids are dense in (chunk, local order)
// of first appearances.  The uniques go to t->uniq[col].
void merge_dicts(FslrTsv *t, int col, std::vector<ChunkDict> &D, int64_t rows, int32_t *codes, int64_t *n_uniq,
                 int64_t *uniq_bytes) {
    const int T = (int)D.size();
    std::vector<std::thread> pool;
    auto run = [&](auto &&f) {
        for (int c = 0; c < T; ++c) pool.emplace_back([&, c] { f(c); });
        for (auto &th : pool) th.join();
        pool.clear();
    };
    std::vector<std::vector<int64_t>> first((size_t)T);   // -1: first appearance; else (chunk << 32 | k)
    std::vector<std::vector<int32_t>> remap((size_t)T);
    run([&](int c) {
        D[(size_t)c].m = StrTable();                      // the local tables are done
        first[(size_t)c].resize(D[(size_t)c].ord.size());
        remap[(size_t)c].resize(D[(size_t)c].ord.size());
    });
    run([&](int sh) {
        StrTable m;
        std::vector<int64_t> where;
        for (int c = 0; c < T; ++c) {
            const auto &ord = D[(size_t)c].ord;
            const auto &oh = D[(size_t)c].oh;
            for (size_t k = 0; k < ord.size(); ++k) {
                if ((int)(oh[k] % (uint64_t)T) != sh) continue;
                const int32_t id = *m.find_or_insert(ord[k], oh[k], (int32_t)where.size());
                if (id == (int32_t)where.size()) {
                    where.push_back(((int64_t)c << 32) | (int64_t)k);
                    first[(size_t)c][k] = -1;
                } else {
                    first[(size_t)c][k] = where[(size_t)id];
                }
            }
        }
    });
    std::vector<int64_t> base((size_t)T + 1, 0);
    for (int c = 0; c < T; ++c)
        base[(size_t)c + 1] = base[(size_t)c] + std::count(first[(size_t)c].begin(), first[(size_t)c].end(), (int64_t)-1);
    std::vector<std::string_view> &order = t->uniq[(size_t)col];
    order.assign((size_t)base[(size_t)T], std::string_view());
    run([&](int c) {
        int64_t id = base[(size_t)c];
        for (size_t k = 0; k < first[(size_t)c].size(); ++k)
            if (first[(size_t)c][k] < 0) { remap[(size_t)c][k] = (int32_t)id; order[(size_t)id++] = D[(size_t)c].ord[k]; }
    });
    run([&](int c) {
        for (size_t k = 0; k < first[(size_t)c].size(); ++k)
            if (first[(size_t)c][k] >= 0) remap[(size_t)c][k] = remap[first[(size_t)c][k] >> 32][first[(size_t)c][k] & 0xffffffff];
        const int64_t a = rows * c / T, e = rows * (c + 1) / T;
        const int32_t *r = remap[(size_t)c].data();
        for (int64_t i = a; i < e; ++i) codes[i] = r[codes[i]];
    });
    int64_t bytes = 0;
    for (auto &sv : order) bytes += (int64_t)sv.size();
    *n_uniq = (int64_t)order.size();
    *uniq_bytes = bytes;
}

// Field starts of the line [s, le): fs[k] = start of field k, fs[count] = le + 1 (so field k is
// [fs[k], fs[k+1] - 1)).  Tabs are found 16 bytes at a time (loads stay inside the line).  Returns
// the field count, or -1 past maxf fields.
inline int split_fields(const char *s, const char *le, const char **fs, int maxf) {
    int k = 0;
    fs[k++] = s;
    const char *p = s;
    const __m128i tab = _mm_set1_epi8('\t');
    for (; p + 16 <= le; p += 16) {
        unsigned m = (unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_loadu_si128((const __m128i *)p), tab));
        while (m) {
            if (k > maxf) return -1;
            fs[k++] = p + __builtin_ctz(m) + 1;
            m &= m - 1;
        }
    }
    for (; p < le; ++p)
        if (*p == '\t') {
            if (k > maxf) return -1;
            fs[k++] = p + 1;
        }
    fs[k] = le + 1;
    return k;
}

inline std::string_view row_field(const FslrTsv *t, int64_t i, int col) {
    const int64_t rows = fslr_tsv_rows(t);
    const char *b = t->data;
    const char *s = b + t->line[i];
    const char *e = b + t->line[rows + 1 + i];
    if (e > s && e[-1] == '\n') --e;
    if (e > s && e[-1] == '\r') --e;
    return field(s, e, col);
}
}  // namespace

extern "C" {

int fslr_tsv_int_column(const FslrTsv *t, int col, int64_t *out) {
    if (col < 0 || col >= (int)t->names.size()) return FSLR_INGEST_ERROR;
    std::atomic<bool> ok{true};
    parallel_for(fslr_tsv_rows(t), t->n_threads, [&](int64_t a, int64_t e, int) {
        for (int64_t i = a; i < e && ok.load(std::memory_order_relaxed); ++i)
            if (!canon_int(row_field(t, i, col), &out[i])) ok = false;
    });
    return ok ? FSLR_INGEST_OK : FSLR_INGEST_DECLINE;
}

int fslr_tsv_int_columns(const FslrTsv *t, int n, const int32_t *cols, int64_t *const *outs) {
    const int ncol = (int)t->names.size();
    int maxc = -1;
    for (int k = 0; k < n; ++k) {
        if (cols[k] < 0 || cols[k] >= ncol) return FSLR_INGEST_ERROR;
        maxc = std::max(maxc, (int)cols[k]);
    }
    if (n == 0) return FSLR_INGEST_OK;
    std::vector<int> slot((size_t)maxc + 1, -1);          // column -> output (one output per column)
    for (int k = 0; k < n; ++k) slot[(size_t)cols[k]] = k;
    const int64_t rows = fslr_tsv_rows(t);
    std::atomic<bool> ok{true};
    const char *b = t->data;
    parallel_for(rows, t->n_threads, [&](int64_t a, int64_t e, int) {
        for (int64_t i = a; i < e && ok.load(std::memory_order_relaxed); ++i) {
            const char *s = b + t->line[i];
            const char *le = b + t->line[rows + 1 + i];
            if (le > s && le[-1] == '\n') --le;
            if (le > s && le[-1] == '\r') --le;
            const char *p = s;
            for (int c = 0; c <= maxc; ++c) {
                const char *q = p ? static_cast<const char *>(std::memchr(p, '\t', (size_t)(le - p))) : nullptr;
                const char *fe = q ? q : le;
                if (slot[(size_t)c] >= 0) {
                    int64_t v;
                    if (!p || !canon_int(std::string_view(p, (size_t)(fe - p)), &v)) { ok = false; break; }
                    outs[slot[(size_t)c]][i] = v;
                }
                p = q ? q + 1 : nullptr;                    // a missing field: NaN in pandas
            }
        }
    });
    return ok ? FSLR_INGEST_OK : FSLR_INGEST_DECLINE;
}

int fslr_tsv_factorize(FslrTsv *t, int col, int32_t *codes, int64_t *n_uniq, int64_t *uniq_bytes) {
    if (col < 0 || col >= (int)t->names.size()) return FSLR_INGEST_ERROR;
    const int64_t rows = fslr_tsv_rows(t);
    const int T = (int)std::min<int64_t>(t->n_threads, std::max<int64_t>(1, rows / 4096));
    std::vector<ChunkDict> D((size_t)T);
    parallel_for(rows, T, [&](int64_t a, int64_t e, int c) {
        ChunkDict &d = D[(size_t)c];
        for (int64_t i = a; i < e && !d.na; ++i) codes[i] = d.add(row_field(t, i, col));
    });
    bool all_int = rows > 0;
    for (auto &d : D) {
        if (d.na) return FSLR_INGEST_DECLINE;
        all_int = all_int && d.all_int;
    }
    if (all_int) return FSLR_INGEST_DECLINE;   // pandas would type the column as int64
    merge_dicts(t, col, D, rows, codes, n_uniq, uniq_bytes);
    return FSLR_INGEST_OK;
}

int fslr_tsv_uniques(const FslrTsv *t, int col, char *buf, int64_t *ends) {
    if (col < 0 || col >= (int)t->names.size()) return FSLR_INGEST_ERROR;
    int64_t off = 0, k = 0;
    for (auto &s : t->uniq[col]) {
        std::memcpy(buf + off, s.data(), s.size());
        off += (int64_t)s.size();
        ends[k++] = off;
    }
    return FSLR_INGEST_OK;
}

}  // extern "C"

// ---- writer: rows copied verbatim + a per-row suffix (main.py:344,351 to_csv) ----
namespace {
// pandas would infer a bool column from these (true_values/false_values defaults, case-insensitive).
bool boolish(std::string_view f) {
    auto eq = [&](const char *w) {
        size_t n = std::strlen(w);
        if (f.size() != n) return false;
        for (size_t i = 0; i < n; ++i)
            if ((f[i] | 0x20) != w[i]) return false;
        return true;
    };
    return eq("true") || eq("false");
}
// Any field pandas' C parser could turn into a number (strtod consumes all of it).  strtod reads
// nothing from a field that starts with a letter other than i / n (inf, infinity, nan) or with
// another character that cannot begin a number, so those fields skip the call.
bool numeric(std::string_view f) {
    if (f.empty()) return false;
    const unsigned char c0 = (unsigned char)f[0];
    const bool may = (c0 >= '0' && c0 <= '9') || c0 == '+' || c0 == '-' || c0 == '.' || c0 == 'i' || c0 == 'I' ||
                     c0 == 'n' || c0 == 'N' || std::isspace(c0);
    if (!may) return false;
    char small[96];
    std::string big;
    const char *z;
    if (f.size() < sizeof(small)) {
        std::memcpy(small, f.data(), f.size());
        small[f.size()] = '\0';
        z = small;
    } else {
        big.assign(f);
        z = big.c_str();
    }
    char *end = nullptr;
    std::strtod(z, &end);
    return end == z + f.size();
}
}  // namespace

extern "C" {

int fslr_tsv_verbatim(const FslrTsv *t) { return fslr_tsv_scan(t, 0, nullptr, nullptr); }

int fslr_tsv_scan(const FslrTsv *t, int n_int, const int32_t *int_cols, int64_t *const *outs) {
    return fslr_tsv_scan_all(const_cast<FslrTsv *>(t), n_int, int_cols, outs, 0, nullptr, nullptr, nullptr);
}

int fslr_tsv_scan_all(FslrTsv *t, int n_int, const int32_t *int_cols, int64_t *const *outs, int n_str,
                      const int32_t *str_cols, int32_t *const *str_codes, int64_t *str_counts) {
    const int ncol = (int)t->names.size();
    const int64_t rows = fslr_tsv_rows(t);
    if (rows == 0) return FSLR_INGEST_DECLINE;
    std::vector<int> slot((size_t)ncol, -1), sslot((size_t)ncol, -1);   // column -> int / string output
    for (int k = 0; k < n_int; ++k) {
        if (int_cols[k] < 0 || int_cols[k] >= ncol) return FSLR_INGEST_ERROR;
        slot[(size_t)int_cols[k]] = k;
    }
    for (int k = 0; k < n_str; ++k) {
        if (str_cols[k] < 0 || str_cols[k] >= ncol || slot[(size_t)str_cols[k]] >= 0) return FSLR_INGEST_ERROR;
        sslot[(size_t)str_cols[k]] = k;
    }
    // pandas renames empty header names ('Unnamed: N') and repeated ones ('x.1'): the input's own
    // header line would then not be what to_csv writes
    {
        std::vector<std::string> nm(t->names.begin(), t->names.end());
        for (const std::string &x : nm)
            if (x.empty()) return FSLR_INGEST_DECLINE;
        std::sort(nm.begin(), nm.end());
        if (std::adjacent_find(nm.begin(), nm.end()) != nm.end()) return FSLR_INGEST_DECLINE;
    }
    // One row-major pass, each line split once.  Every row must hold exactly ncol fields: a longer
    // row makes pandas raise (or index by the first column), a shorter one NaN-fills — either way
    // the row bytes are not what to_csv writes.  Per column: all fields canonical ints (pandas
    // types it int64, the text round-trips), or text with no numeric-looking, bool-looking or
    // non-empty NA field and at least one text field (empty fields come back as '' either way).
    // Requested int columns are parsed, requested string columns factorized, in the same pass.
    std::atomic<int> bad{0};
    const auto t_start = std::chrono::steady_clock::now();
    const int T = (int)std::min<int64_t>(t->n_threads, std::max<int64_t>(1, rows / 4096));
    std::vector<std::vector<unsigned char>> st((size_t)T, std::vector<unsigned char>((size_t)ncol * 3, 0));
    std::vector<std::vector<ChunkDict>> D((size_t)n_str, std::vector<ChunkDict>((size_t)T));
    const char *b = t->data;
    parallel_for(rows, T, [&](int64_t a, int64_t e, int w) {
        // per column: ai = every field so far a canonical int, tk = no field rules text out, at = a text field
        std::vector<unsigned char> ai((size_t)ncol, 1), tk((size_t)ncol, 1), at((size_t)ncol, 0);
        // the previous row's field per column and its class (bit 0: canonical int, bit 1: rules text
        // out): columns such as strand or version repeat one value, which is classified once
        std::vector<std::string_view> prev((size_t)ncol);
        std::vector<unsigned char> pcls((size_t)ncol, 0);
        std::vector<const char *> fs((size_t)ncol + 2);
        // per column: the requested int output, the requested string codes and dictionary (raw
        // pointers held in locals: the byte stores below may alias anything held in memory)
        std::vector<int64_t *> iout((size_t)ncol, nullptr);
        std::vector<int32_t *> sout((size_t)ncol, nullptr);
        std::vector<ChunkDict *> dict((size_t)ncol, nullptr);
        for (int c = 0; c < ncol; ++c) {
            if (slot[(size_t)c] >= 0) iout[(size_t)c] = outs[slot[(size_t)c]];
            if (sslot[(size_t)c] >= 0) {
                sout[(size_t)c] = str_codes[sslot[(size_t)c]];
                dict[(size_t)c] = &D[(size_t)sslot[(size_t)c]][(size_t)w];
            }
        }
        unsigned char *const AI = ai.data(), *const TK = tk.data(), *const AT = at.data(), *const PC = pcls.data();
        std::string_view *const PV = prev.data();
        const char **const FS = fs.data();
        int64_t *const *const IO = iout.data();
        int32_t *const *const SO = sout.data();
        ChunkDict *const *const DI = dict.data();
        const int64_t *const L0 = t->line.data(), *const L1 = L0 + rows + 1;
        for (int64_t i = a; i < e && !bad.load(std::memory_order_relaxed); ++i) {
            const char *s = b + L0[i];
            const char *le = b + L1[i];
            if (le > s && le[-1] == '\n') --le;
            if (le > s && le[-1] == '\r') --le;
            if (split_fields(s, le, FS, ncol) != ncol) { bad = 1; break; }   // ragged row
            for (int c = 0; c < ncol; ++c) {
                const std::string_view f(FS[c], (size_t)(FS[c + 1] - 1 - FS[c]));
                if (int64_t *const io = IO[c]) {
                    // a requested int column: every field a canonical int (its class stays int)
                    int64_t v;
                    if (!canon_int(f, &v)) { bad = 1; break; }
                    io[i] = v;
                    continue;
                }
                unsigned char cls;
                if (i > a && !(PC[c] & 1) && f == PV[c]) {
                    cls = PC[c];
                } else {
                    int64_t v = 0;
                    cls = canon_int(f, &v) ? 1 : 0;
                    if (!cls && !f.empty() && (is_na(f) || boolish(f) || numeric(f))) cls |= 2;
                    PV[c] = f;
                    PC[c] = cls;
                }
                if (ChunkDict *const d = DI[c]) {
                    SO[c][i] = d->add(f);
                    if (d->na) { bad = 1; break; }
                }
                if (AI[c] && !(cls & 1)) {
                    AI[c] = 0;
                    if (i > a) TK[c] = 0;          // the earlier fields were canonical ints: numeric text
                }
                if (!AI[c] && !f.empty() && TK[c]) {
                    if (cls & 2) TK[c] = 0;
                    else AT[c] = 1;
                }
                if (!AI[c] && !TK[c]) { bad = 1; break; }    // neither int nor text: decline
            }
        }
        auto &o = st[(size_t)w];
        for (int c = 0; c < ncol; ++c) { o[(size_t)c] = ai[(size_t)c]; o[(size_t)(ncol + c)] = tk[(size_t)c]; o[(size_t)(2 * ncol + c)] = at[(size_t)c]; }
    });
    if (bad) return FSLR_INGEST_DECLINE;
    const auto t_scan = std::chrono::steady_clock::now();
    for (int c = 0; c < ncol; ++c) {
        bool all_int = true, text_ok = true, any_text = false;
        for (int w = 0; w < T; ++w) {
            all_int = all_int && st[(size_t)w][(size_t)c];
            text_ok = text_ok && !st[(size_t)w][(size_t)c] && st[(size_t)w][(size_t)(ncol + c)];   // an all-int chunk is numeric
            any_text = any_text || st[(size_t)w][(size_t)(2 * ncol + c)];
        }
        if (all_int) {
            if (sslot[(size_t)c] >= 0) return FSLR_INGEST_DECLINE;      // pandas types it int64, not text
            continue;
        }
        if (!(text_ok && any_text)) return FSLR_INGEST_DECLINE;
    }
    for (int k = 0; k < n_str; ++k)
        merge_dicts(t, str_cols[k], D[(size_t)k], rows, str_codes[k], &str_counts[2 * k], &str_counts[2 * k + 1]);
    if (std::getenv("FSLR_INGEST_TIMING"))
        std::fprintf(stderr, "fslr_tsv_scan_all: rows %lld threads %d scan %.3f s merge %.3f s\n", (long long)rows, T,
                     std::chrono::duration<double>(t_scan - t_start).count(),
                     std::chrono::duration<double>(std::chrono::steady_clock::now() - t_scan).count());
    return FSLR_INGEST_OK;
}

int fslr_tsv_write(const FslrTsv *t, const char *path, const char *header_suffix, const int64_t *rows_out,
                   int64_t n_out, const int32_t *suffix_id, const char *suffix_buf, const int64_t *suffix_ends,
                   char *err, size_t errlen) {
    // Each thread owns a contiguous range of output rows: their byte lengths are summed first, so
    // every range knows its file offset and is formatted and written (pwrite) independently.
    const int fd = ::open(path, O_WRONLY | O_CREAT | O_TRUNC, 0666);
    if (fd < 0) { set_err(err, errlen, std::string("cannot write ") + path); return FSLR_INGEST_ERROR; }
    std::string head;
    for (size_t c = 0; c < t->names.size(); ++c) { if (c) head += '\t'; head += t->names[c]; }
    head += header_suffix;
    head += '\n';
    const int64_t rows = fslr_tsv_rows(t);
    const char *b = t->data;
    auto span = [&](int64_t i, const char **s) {
        *s = b + t->line[i];
        const char *le = b + t->line[rows + 1 + i];
        if (le > *s && le[-1] == '\n') --le;
        if (le > *s && le[-1] == '\r') --le;
        return (int64_t)(le - *s);
    };
    auto sfx = [&](int64_t k, int64_t *ss) {
        const int32_t u = suffix_id[k];
        *ss = u ? suffix_ends[u - 1] : 0;
        return suffix_ends[u] - *ss;
    };
    const int T = (int)std::min<int64_t>(std::max(1, t->n_threads), std::max<int64_t>(1, n_out / 4096));
    std::vector<int64_t> bytes((size_t)T + 1, 0);
    std::atomic<bool> oob{false}, werr{false};
    auto range = [&](int w) { return std::make_pair(n_out * w / T, n_out * (w + 1) / T); };
    {
        std::vector<std::thread> pool;
        for (int w = 0; w < T; ++w)
            pool.emplace_back([&, w] {
                auto [a, e] = range(w);
                int64_t tot = 0;
                for (int64_t k = a; k < e; ++k) {
                    const int64_t i = rows_out[k];
                    if (i < 0 || i >= rows) { oob = true; return; }
                    const char *s;
                    int64_t ss;
                    tot += span(i, &s) + sfx(k, &ss) + 1;
                }
                bytes[(size_t)w + 1] = tot;
            });
        for (auto &th : pool) th.join();
    }
    if (oob) { ::close(fd); set_err(err, errlen, "row index out of range"); return FSLR_INGEST_ERROR; }
    bytes[0] = (int64_t)head.size();
    for (int w = 0; w < T; ++w) bytes[(size_t)w + 1] += bytes[(size_t)w];
    // The file is sized once and mapped: each thread copies its rows into its own byte range.  Page
    // faults on a shared file mapping run in parallel, where buffered pwrite()s of one file serialise
    // on its inode lock (a 16-thread writer ran at one thread's copy speed).  pwrite() stays the
    // fallback when the mapping is refused.
    const int64_t total = bytes[(size_t)T];
    // the blocks are reserved first (a full disk is an error here, not a SIGBUS in a mapped store)
    const int fa = total > 0 ? ::posix_fallocate(fd, 0, (off_t)total) : 0;
    if (fa != 0 && fa != EOPNOTSUPP && fa != EINVAL) {
        ::close(fd);
        set_err(err, errlen, std::string("cannot write ") + path + ": " + std::strerror(fa));
        return FSLR_INGEST_ERROR;
    }
    if (total > 0 && fa == 0 && ::ftruncate(fd, (off_t)total) == 0) {
        void *m = ::mmap(nullptr, (size_t)total, PROT_WRITE, MAP_SHARED, fd, 0);
        if (m != MAP_FAILED) {
            char *out = static_cast<char *>(m);
            std::memcpy(out, head.data(), head.size());
            std::vector<std::thread> pool;
            for (int w = 0; w < T; ++w)
                pool.emplace_back([&, w] {
                    auto [a, e] = range(w);
                    char *o = out + bytes[(size_t)w];
                    for (int64_t k = a; k < e; ++k) {
                        const char *s;
                        int64_t ss;
                        const int64_t ln = span(rows_out[k], &s);
                        std::memcpy(o, s, (size_t)ln);
                        o += ln;
                        const int64_t sl = sfx(k, &ss);
                        std::memcpy(o, suffix_buf + ss, (size_t)sl);
                        o += sl;
                        *o++ = '\n';
                    }
                });
            for (auto &th : pool) th.join();
            const bool ok = ::munmap(m, (size_t)total) == 0;
            if (::close(fd) != 0 || !ok) {
                set_err(err, errlen, "write failed");
                return FSLR_INGEST_ERROR;
            }
            return FSLR_INGEST_OK;
        }
    }
    auto put = [&](const char *p, size_t len, int64_t off) {
        while (len) {
            const ssize_t r = ::pwrite(fd, p, len, off);
            if (r <= 0) { werr = true; return; }
            p += r;
            len -= (size_t)r;
            off += r;
        }
    };
    put(head.data(), head.size(), 0);
    {
        std::vector<std::thread> pool;
        for (int w = 0; w < T; ++w)
            pool.emplace_back([&, w] {
                auto [a, e] = range(w);
                int64_t off = bytes[(size_t)w];
                std::string o;
                o.reserve(8 << 20);
                for (int64_t k = a; k < e && !werr; ++k) {
                    const char *s;
                    int64_t ss;
                    const int64_t ln = span(rows_out[k], &s);
                    o.append(s, (size_t)ln);
                    const int64_t sl = sfx(k, &ss);
                    o.append(suffix_buf + ss, (size_t)sl);
                    o += '\n';
                    if (o.size() >= (8u << 20) || k + 1 == e) {
                        put(o.data(), o.size(), off);
                        off += (int64_t)o.size();
                        o.clear();
                    }
                }
            });
        for (auto &th : pool) th.join();
    }
    if (::close(fd) != 0 || werr) {
        set_err(err, errlen, "write failed");
        return FSLR_INGEST_ERROR;
    }
    return FSLR_INGEST_OK;
}

}  // extern "C"

// ---- suffix text: the numbers DataFrame.to_csv appends (cluster, n_reads, avg_alignment_score) ----
// pandas writes an int64 value as its decimal text and a float64 value as numpy's str() of it
// (get_values_for_csv: values.astype(str) when float_format is None), i.e. Python's repr: the
// shortest digits that round-trip, positional for decimal exponents -4 <= x < 16 (with ".0" when
// integral), otherwise d[.ddd]e+XX.  std::to_chars gives the shortest round-trip digits.

namespace {

int repr_double(double v, char *out) {
  char sci[64];
  auto r = std::to_chars(sci, sci + sizeof(sci), v, std::chars_format::scientific);
  if (r.ec != std::errc()) return -1;
  const char *p = sci;
  const char *end = r.ptr;
  char *o = out;
  if (*p == '-') *o++ = *p++;
  std::string digits;
  const char *e = std::find(p, end, 'e');
  for (const char *q = p; q < e; ++q)
    if (*q != '.') digits.push_back(*q);
  const int x = std::atoi(std::string(e + 1, end).c_str());        // v = d.ddd x 10^x
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  const int nd = static_cast<int>(digits.size());
  if (x >= -4 && x < 16) {
    const int decpt = x + 1;                                           // digits before the point
    if (decpt <= 0) {
      *o++ = '0';
      *o++ = '.';
      for (int k = 0; k < -decpt; ++k) *o++ = '0';
      for (char c : digits) *o++ = c;
    } else if (decpt >= nd) {
      for (char c : digits) *o++ = c;
      for (int k = nd; k < decpt; ++k) *o++ = '0';
      *o++ = '.';
      *o++ = '0';
    } else {
      for (int k = 0; k < nd; ++k) {
        if (k == decpt) *o++ = '.';
        *o++ = digits[k];
      }
    }
  } else {
    *o++ = digits[0];
    if (nd > 1) {
      *o++ = '.';
      for (int k = 1; k < nd; ++k) *o++ = digits[k];
    }
    *o++ = 'e';
    *o++ = x < 0 ? '-' : '+';
    const int ax = x < 0 ? -x : x;
    if (ax < 10) *o++ = '0';
    o += std::sprintf(o, "%d", ax);
  }
  return static_cast<int>(o - out);
}

}  // namespace

extern "C" {

int fslr_format_suffix(int n_cols, const int32_t *kinds, const void *const *cols, int64_t n_keys, char *out,
                       int64_t cap, int64_t *ends) {
  if (n_cols < 0 || n_keys < 0 || (!out && cap) || (n_keys && !ends)) return FSLR_INGEST_ERROR;
  for (int c = 0; c < n_cols; ++c)
    if (kinds[c] != 0 && kinds[c] != 1) return FSLR_INGEST_ERROR;
  // key ranges formatted by threads into their own buffers, then placed by a prefix sum
  const char *env = std::getenv("OMP_NUM_THREADS");
  int T = env ? std::atoi(env) : 0;
  if (T <= 0) T = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  T = (int)std::min<int64_t>(T, std::max<int64_t>(1, n_keys / 8192));
  std::vector<std::string> part((size_t)T);
  std::atomic<int> rc{FSLR_INGEST_OK};
  parallel_for(n_keys, T, [&](int64_t a, int64_t e, int w) {
    std::string &o = part[(size_t)w];
    o.reserve((size_t)(e - a) * (size_t)n_cols * 12);
    char tmp[64];
    for (int64_t k = a; k < e; ++k) {
      for (int c = 0; c < n_cols; ++c) {
        int len;
        if (kinds[c] == 0) {
          len = std::sprintf(tmp, "%lld", static_cast<long long>(static_cast<const int64_t *>(cols[c])[k]));
        } else {
          const double v = static_cast<const double *>(cols[c])[k];
          if (!std::isfinite(v)) { rc = FSLR_INGEST_DECLINE; return; }     // NaN / inf: pandas' own text
          len = repr_double(v, tmp);
          if (len < 0) { rc = FSLR_INGEST_ERROR; return; }
        }
        o += '\t';
        o.append(tmp, (size_t)len);
      }
      ends[k] = (int64_t)o.size();                 // local for now
    }
  });
  if (rc != FSLR_INGEST_OK) return rc;
  std::vector<int64_t> base((size_t)T + 1, 0);
  for (int w = 0; w < T; ++w) base[(size_t)w + 1] = base[(size_t)w] + (int64_t)part[(size_t)w].size();
  if (base[(size_t)T] > cap) return FSLR_INGEST_ERROR;
  parallel_for(n_keys, T, [&](int64_t a, int64_t e, int w) {
    std::memcpy(out + base[(size_t)w], part[(size_t)w].data(), part[(size_t)w].size());
    for (int64_t k = a; k < e; ++k) ends[k] += base[(size_t)w];
  });
  return FSLR_INGEST_OK;
}

}  // extern "C"

// ---- CSR grouping of the prepared interval list (prepare_data order -> reads by rank) ----
extern "C" {

int fslr_group_by_first_appearance(const int64_t *codes, int64_t n, int64_t n_codes, int64_t *read_code,
                                   int64_t *n_reads, int64_t *off, int64_t *perm) {
  if (n < 0 || n_codes < 0 || (n && (!codes || !perm)) || !n_reads || !off) return FSLR_INGEST_ERROR;
  const char *env = std::getenv("OMP_NUM_THREADS");
  int T = env ? std::atoi(env) : 0;
  if (T <= 0) T = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  T = (int)std::min<int64_t>(T, std::max<int64_t>(1, n / 65536));
  // 1. each code's first position (rank = order of first appearance, cluster.py:189-191)
  std::vector<std::atomic<int64_t>> first_at(static_cast<size_t>(n_codes));
  parallel_for(n_codes, T, [&](int64_t a, int64_t e, int) {
    for (int64_t c = a; c < e; ++c) first_at[(size_t)c].store(n, std::memory_order_relaxed);
  });
  std::atomic<bool> bad{false};
  parallel_for(n, T, [&](int64_t a, int64_t e, int) {
    for (int64_t k = a; k < e; ++k) {
      const int64_t c = codes[k];
      if (c < 0 || c >= n_codes) { bad = true; return; }
      int64_t cur = first_at[(size_t)c].load(std::memory_order_relaxed);
      while (k < cur && !first_at[(size_t)c].compare_exchange_weak(cur, k, std::memory_order_relaxed)) {}
    }
  });
  if (bad) return FSLR_INGEST_ERROR;
  // 2. ranks: a position is a rank start when it is its code's first; prefix over positions
  std::vector<int64_t> rk(static_cast<size_t>(n));            // first-position flags, then the rank per position
  std::vector<int64_t> base((size_t)T + 1, 0);
  parallel_for(n, T, [&](int64_t a, int64_t e, int w) {
    int64_t cnt = 0;
    for (int64_t k = a; k < e; ++k) cnt += first_at[(size_t)codes[k]].load(std::memory_order_relaxed) == k;
    base[(size_t)w + 1] = cnt;
  });
  for (int w = 0; w < T; ++w) base[(size_t)w + 1] += base[(size_t)w];
  const int64_t nr = base[(size_t)T];
  std::vector<int64_t> rank_of(static_cast<size_t>(n_codes), -1);
  parallel_for(n, T, [&](int64_t a, int64_t e, int w) {
    int64_t r = base[(size_t)w];
    for (int64_t k = a; k < e; ++k) {
      const int64_t c = codes[k];
      if (first_at[(size_t)c].load(std::memory_order_relaxed) == k) { rank_of[(size_t)c] = r; read_code[r] = c; ++r; }
    }
  });
  // 3. rank per position and counts per rank
  std::vector<std::atomic<int64_t>> cnt(static_cast<size_t>(nr) + 1);
  parallel_for(nr + 1, T, [&](int64_t a, int64_t e, int) {
    for (int64_t r = a; r < e; ++r) cnt[(size_t)r].store(0, std::memory_order_relaxed);
  });
  parallel_for(n, T, [&](int64_t a, int64_t e, int) {
    for (int64_t k = a; k < e; ++k) {
      const int64_t r = rank_of[(size_t)codes[k]];
      rk[(size_t)k] = r;
      cnt[(size_t)r + 1].fetch_add(1, std::memory_order_relaxed);
    }
  });
  off[0] = 0;
  for (int64_t r = 0; r < nr; ++r) off[r + 1] = off[r] + cnt[(size_t)r + 1].load(std::memory_order_relaxed);
  // 4. stable scatter (data order inside a read): thread w owns a contiguous range of ranks holding
  // about n / T positions and walks every position, keeping its own
  std::vector<int64_t> rb((size_t)T + 1, nr);
  rb[0] = 0;
  for (int w = 1; w < T; ++w) rb[(size_t)w] = std::upper_bound(off, off + nr + 1, n * w / T) - off - 1;
  for (int w = 1; w <= T; ++w) rb[(size_t)w] = std::max(rb[(size_t)w], rb[(size_t)w - 1]);
  std::vector<std::thread> pool;
  for (int w = 0; w < T; ++w)
    pool.emplace_back([&, w] {
      const int64_t r0 = rb[(size_t)w], r1 = rb[(size_t)w + 1];
      if (r0 >= r1) return;
      std::vector<int64_t> cur(off + r0, off + r1);
      for (int64_t k = 0; k < n; ++k) {
        const int64_t r = rk[(size_t)k];
        if (r >= r0 && r < r1) perm[cur[(size_t)(r - r0)]++] = k;
      }
    });
  for (auto &th : pool) th.join();
  *n_reads = nr;
  return FSLR_INGEST_OK;
}

}  // extern "C"

// ---- threaded gather of several int64 columns by one index (prepare_data's sort + mask) ----
extern "C" {

int fslr_gather_i64(int n_arrays, const int64_t *const *src, int64_t *const *dst, const int64_t *idx, int64_t n,
                    int n_threads) {
  if (n_arrays < 0 || n < 0 || (n && !idx)) return FSLR_INGEST_ERROR;
  const int64_t per = 1 << 16;
  const int64_t chunks = (n + per - 1) / per;
  int t = n_threads > 0 ? n_threads : static_cast<int>(std::thread::hardware_concurrency());
  t = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>({static_cast<int64_t>(t), chunks, 64})));
  std::atomic<int64_t> next{0};
  auto work = [&]() {
    for (int64_t c; (c = next.fetch_add(1)) < chunks;) {
      const int64_t b = c * per, e = std::min(n, b + per);
      for (int a = 0; a < n_arrays; ++a) {
        const int64_t *s = src[a];
        int64_t *d = dst[a];
        for (int64_t k = b; k < e; ++k) d[k] = s[idx[k]];
      }
    }
  };
  std::vector<std::thread> pool;
  for (int k = 1; k < t; ++k) pool.emplace_back(work);
  work();
  for (auto &th : pool) th.join();
  return FSLR_INGEST_OK;
}

}  // extern "C"

// ---- keep_fillings + prepare_data's per-row columns (fastcli) ----
extern "C" {

int fslr_fillings(int64_t n_rows, const int32_t *qcode, int64_t n_q, const uint8_t *row_keep, const int64_t *rstart,
                  const int64_t *rend, const int64_t *aln, const int64_t *qstart, const int64_t *qend,
                  const int64_t *nal, const int32_t *ccode, const int64_t *chrom_lut, int64_t *n_out, int64_t *frow,
                  int64_t *start, int64_t *end, int64_t *aln_o, int64_t *qc_o, int64_t *nal_o, int64_t *qlen2_o,
                  int64_t *chrom_o, int n_threads) {
    if (n_rows < 0 || n_q < 0 || !qcode || !n_out) return FSLR_INGEST_ERROR;
    int T = n_threads > 0 ? n_threads : (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    T = (int)std::min<int64_t>(T, std::max<int64_t>(1, n_rows / 65536));
    // 1. first and last row (file order, rows kept by row_keep) of every qname, and 2. qlen2 =
    // max(qend) - min(qstart) over its fillings (cluster.py:14-31).  A file grouped by qname (the
    // mapping step writes it so) has each qname's rows as one run: runs are found and measured in
    // parallel; any other file takes the ordered pass
    std::vector<int64_t> first((size_t)n_q, -1), last((size_t)n_q, -1);
    std::vector<int64_t> lo((size_t)n_q, INT64_MAX), hi((size_t)n_q, INT64_MIN);
    std::atomic<bool> bad{false}, grouped{true};
    {
        std::unique_ptr<std::atomic<int8_t>[]> seen(new std::atomic<int8_t>[(size_t)n_q]);
        parallel_for(n_q, T, [&](int64_t a, int64_t e, int) {
            for (int64_t q = a; q < e; ++q) seen[q].store(0, std::memory_order_relaxed);
        });
        parallel_for(n_rows, T, [&](int64_t a, int64_t e, int) {
            for (int64_t i = a; i < e && !bad && grouped; ++i) {
                const int32_t q = qcode[i];
                if (q < 0 || q >= n_q) { bad = true; return; }
                if (i > 0 && qcode[i - 1] == q) continue;             // not a run start
                if (seen[q].exchange(1, std::memory_order_relaxed)) { grouped = false; return; }
                int64_t j = i + 1;
                while (j < n_rows && qcode[j] == q) ++j;
                if (row_keep && !row_keep[i]) {                       // delete_false drops whole qnames
                    for (int64_t k = i; k < j; ++k)
                        if (row_keep[k]) { grouped = false; return; }
                    continue;
                }
                for (int64_t k = i; k < j; ++k)
                    if (row_keep && !row_keep[k]) { grouped = false; return; }
                first[(size_t)q] = i;
                last[(size_t)q] = j - 1;
                int64_t l = INT64_MAX, h = INT64_MIN;
                for (int64_t k = i + 1; k < j - 1; ++k) {
                    l = std::min(l, qstart[k]);
                    h = std::max(h, qend[k]);
                }
                lo[(size_t)q] = l;
                hi[(size_t)q] = h;
            }
        });
    }
    if (bad) return FSLR_INGEST_ERROR;
    if (!grouped) {
        std::fill(first.begin(), first.end(), -1);
        std::fill(last.begin(), last.end(), -1);
        for (int64_t i = 0; i < n_rows; ++i) {
            if (row_keep && !row_keep[i]) continue;
            const int32_t q = qcode[i];
            if (q < 0 || q >= n_q) return FSLR_INGEST_ERROR;
            if (first[(size_t)q] < 0) first[(size_t)q] = i;
            last[(size_t)q] = i;
        }
    }
    auto kept = [&](int64_t i) {
        if (row_keep && !row_keep[i]) return false;
        const int32_t q = qcode[i];
        return first[(size_t)q] != i && last[(size_t)q] != i;
    };
    if (!grouped) {
        std::fill(lo.begin(), lo.end(), INT64_MAX);
        std::fill(hi.begin(), hi.end(), INT64_MIN);
        for (int64_t i = 0; i < n_rows; ++i) {
            if (!kept(i)) continue;
            const int32_t q = qcode[i];
            lo[(size_t)q] = std::min(lo[(size_t)q], qstart[i]);
            hi[(size_t)q] = std::max(hi[(size_t)q], qend[i]);
        }
    }
    // 3. the fillings' columns, compacted in file order
    std::vector<int64_t> base((size_t)T + 1, 0);
    parallel_for(n_rows, T, [&](int64_t a, int64_t e, int w) {
        int64_t c = 0;
        for (int64_t i = a; i < e; ++i) c += kept(i);
        base[(size_t)w + 1] = c;
    });
    for (int w = 0; w < T; ++w) base[(size_t)w + 1] += base[(size_t)w];
    parallel_for(n_rows, T, [&](int64_t a, int64_t e, int w) {
        int64_t k = base[(size_t)w];
        for (int64_t i = a; i < e; ++i) {
            if (!kept(i)) continue;
            const int32_t q = qcode[i];
            frow[k] = i;
            start[k] = std::min(rstart[i], rend[i]);
            end[k] = std::max(rstart[i], rend[i]);
            aln_o[k] = aln[i];
            qc_o[k] = q;
            nal_o[k] = nal[i];
            qlen2_o[k] = hi[(size_t)q] - lo[(size_t)q];
            chrom_o[k] = chrom_lut[ccode[i]];
            ++k;
        }
    });
    *n_out = base[(size_t)T];
    return FSLR_INGEST_OK;
}

}  // extern "C"

// ---- prepare_data's start order when every start is distinct (cluster.py:114) ----------------------
// df.sort_values('start') is numpy's quicksort argsort (pandas nargsort): its order of tied starts is
// the algorithm's own.  When no two starts tie every sort gives the one order, so a stable parallel
// LSD radix sort of (start - min, row) stands in; a tie is reported and the caller sorts with numpy.
extern "C" {

int fslr_argsort_distinct(const int64_t *keys, int64_t n, int64_t *order, int n_threads) {
    if (n < 0 || (n && (!keys || !order))) return -2;
    if (n >= (int64_t(1) << 32)) return -1;
    int T = n_threads;
    if (T <= 0) T = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    T = (int)std::min<int64_t>(T, std::max<int64_t>(1, n / 65536));
    if (n == 0) return 1;
    std::vector<int64_t> lo((size_t)T, INT64_MAX), hi((size_t)T, INT64_MIN);
    parallel_for(n, T, [&](int64_t a, int64_t e, int w) {
        int64_t l = INT64_MAX, h = INT64_MIN;
        for (int64_t i = a; i < e; ++i) {
            l = std::min(l, keys[i]);
            h = std::max(h, keys[i]);
        }
        lo[(size_t)w] = l;
        hi[(size_t)w] = h;
    });
    const int64_t mn = *std::min_element(lo.begin(), lo.end()), mx = *std::max_element(hi.begin(), hi.end());
    if ((uint64_t)mx - (uint64_t)mn >= (uint64_t(1) << 32)) return -1;
    const uint64_t range = (uint64_t)mx - (uint64_t)mn;
    int bits = 0;
    while (bits < 32 && (range >> bits)) ++bits;
    // (key - min) << 32 | row, sorted on bits 32 .. 32 + bits in digits of up to 11 bits
    // uninitialised (a value-initialised vector zero-fills 2 x 8 B x n on one thread first)
    std::unique_ptr<uint64_t[]> vb(new uint64_t[(size_t)n]), tb(new uint64_t[(size_t)n]);
    uint64_t *v = vb.get(), *t = tb.get();
    parallel_for(n, T, [&](int64_t a, int64_t e, int) {
        for (int64_t i = a; i < e; ++i) v[i] = ((uint64_t)(keys[i] - mn) << 32) | (uint64_t)i;
    });
    constexpr int kD = 11, kB = 1 << kD;
    const int passes = (bits + kD - 1) / kD;
    std::vector<int64_t> cnt((size_t)T * kB);
    for (int ps = 0; ps < passes; ++ps) {
        const int sh = 32 + ps * kD;
        std::fill(cnt.begin(), cnt.end(), 0);
        parallel_for(n, T, [&](int64_t a, int64_t e, int w) {
            int64_t *c = cnt.data() + (size_t)w * kB;
            for (int64_t i = a; i < e; ++i) c[(v[i] >> sh) & (kB - 1)]++;
        });
        // digit-major, then slice order: stable
        int64_t acc = 0;
        for (int d = 0; d < kB; ++d)
            for (int w = 0; w < T; ++w) {
                const int64_t x = cnt[(size_t)w * kB + d];
                cnt[(size_t)w * kB + d] = acc;
                acc += x;
            }
        parallel_for(n, T, [&](int64_t a, int64_t e, int w) {
            int64_t *c = cnt.data() + (size_t)w * kB;
            for (int64_t i = a; i < e; ++i) {
                const uint64_t x = v[i];
                t[c[(x >> sh) & (kB - 1)]++] = x;
            }
        });
        std::swap(v, t);
    }
    std::vector<char> tie((size_t)T, 0);
    parallel_for(n, T, [&](int64_t a, int64_t e, int w) {
        bool any = false;
        for (int64_t i = a; i < e; ++i) {
            const uint64_t x = v[i];
            if (i > 0 && (x >> 32) == (v[i - 1] >> 32)) any = true;
            order[i] = (int64_t)(x & 0xFFFFFFFFu);
        }
        tie[(size_t)w] = any;
    });
    for (char c : tie)
        if (c) return 0;
    return 1;
}

}  // extern "C"

