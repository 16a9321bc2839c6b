// ingest.cpp — threaded reader for `{name}.mappings.bed` (include/fslr_ingest.h).
// Host-only C++17; built with g++ into fslr_amd/libfslr_ingest.so.
//
// Layout: the file is read whole into one buffer; line starts are found by a
// per-thread newline count + prefix sum; a column is produced by re-walking each
// line to its k-th tab (the file stays hot in the CPU caches per chunk, and only
// the requested columns are ever materialised).
#include "fslr_ingest.h"

#include <algorithm>
#include <charconv>
#include <cmath>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

struct FslrTsv {
    std::string buf;                      // file contents
    std::vector<int64_t> line;            // [rows starts | file size | rows ends] (header excluded)
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
    static const char *na[] = {"", "#N/A", "#N/A N/A", "#NA", "-1.#IND", "-1.#QNAN", "-NaN", "-nan",
                               "1.#IND", "1.#QNAN", "<NA>", "N/A", "NA", "NULL", "NaN", "None",
                               "n/a", "nan", "null"};
    if (!f.data()) return true;
    for (const char *s : na)
        if (f == s) return true;
    return false;
}

}  // namespace

extern "C" {

int fslr_tsv_open(const char *path, int n_threads, FslrTsv **out, char *err, size_t errlen) {
    *out = nullptr;
    FILE *fp = std::fopen(path, "rb");
    if (!fp) { set_err(err, errlen, std::string("cannot open ") + path); return FSLR_INGEST_ERROR; }
    auto *t = new FslrTsv();
    std::fseek(fp, 0, SEEK_END);
    long sz = std::ftell(fp);
    std::fseek(fp, 0, SEEK_SET);
    t->buf.resize((size_t)std::max(0L, sz));
    size_t got = sz > 0 ? std::fread(&t->buf[0], 1, (size_t)sz, fp) : 0;
    std::fclose(fp);
    if ((long)got != sz) { delete t; set_err(err, errlen, "short read"); return FSLR_INGEST_ERROR; }
    if (n_threads <= 0) {   // the CPU share, not the whole machine: OMP_NUM_THREADS, else min(cores, 16)
        const char *env = std::getenv("OMP_NUM_THREADS");
        n_threads = env ? std::atoi(env) : 0;
        if (n_threads <= 0) n_threads = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    }
    t->n_threads = std::min(n_threads, 256);
    const char *b = t->buf.data();
    const int64_t n = (int64_t)t->buf.size();
    if (std::memchr(b, '"', (size_t)n)) { delete t; set_err(err, errlen, "quoted fields"); return FSLR_INGEST_DECLINE; }
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
    // line starts: count per chunk, prefix, fill. Blank lines are skipped (skip_blank_lines=True).
    const int T = t->n_threads;
    const int64_t len = n - body;
    std::vector<int64_t> cnt(T + 1, 0);
    auto chunk = [&](int i) { return std::make_pair(body + len * i / T, body + len * (i + 1) / T); };
    auto nonblank = [&](int64_t p) {   // p (a line start) begins a non-blank line
        return p < n && !(b[p] == '\n' || (b[p] == '\r' && (p + 1 >= n || b[p + 1] == '\n')));
    };
    // f(p) for every non-blank line start p in [a, e): body itself, and one past each '\n' (memchr scan).
    auto for_starts = [&](int64_t a, int64_t e, auto &&f) {
        if (a >= e) return;
        if (a == body && nonblank(a)) f(a);
        int64_t x = a == body ? a : a - 1;   // a newline at a-1 makes a a start
        while (x < e - 1) {
            const void *q = std::memchr(b + x, '\n', (size_t)(e - 1 - x));
            if (!q) break;
            int64_t p = (int64_t)((const char *)q - b) + 1;
            if (nonblank(p)) f(p);
            x = p;
        }
    };
    std::vector<std::thread> pool;
    for (int i = 0; i < T; ++i)
        pool.emplace_back([&, i] {
            auto [a, e] = chunk(i);
            int64_t c = 0;
            for_starts(a, e, [&](int64_t) { ++c; });
            cnt[i + 1] = c;
        });
    for (auto &th : pool) th.join();
    pool.clear();
    for (int i = 0; i < T; ++i) cnt[i + 1] += cnt[i];
    t->line.resize((size_t)cnt[T] + 1);
    for (int i = 0; i < T; ++i)
        pool.emplace_back([&, i] {
            auto [a, e] = chunk(i);
            int64_t k = cnt[i];
            for_starts(a, e, [&](int64_t p) { t->line[k++] = p; });
        });
    for (auto &th : pool) th.join();
    // Each line ends at its own first newline (blank lines between data lines are skipped,
    // so the next start is not the end). Layout: line[0..rows) starts, line[rows] = n,
    // line[rows+1 .. 2*rows] ends.
    const int64_t rows = cnt[T];
    std::vector<int64_t> ends((size_t)rows);
    parallel_for(rows, T, [&](int64_t a, int64_t e, int) {
        for (int64_t i = a; i < e; ++i) {
            const void *q = std::memchr(b + t->line[i], '\n', (size_t)(n - t->line[i]));
            ends[i] = q ? (int64_t)((const char *)q - b) + 1 : n;
        }
    });
    t->line.resize((size_t)rows * 2 + 1);
    std::copy(ends.begin(), ends.end(), t->line.begin() + rows + 1);
    t->line[rows] = n;
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
inline std::string_view row_field(const FslrTsv *t, int64_t i, int col) {
    const int64_t rows = fslr_tsv_rows(t);
    const char *b = t->buf.data();
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

int fslr_tsv_factorize(FslrTsv *t, int col, int32_t *codes, int64_t *n_uniq, int64_t *uniq_bytes) {
    if (col < 0 || col >= (int)t->names.size()) return FSLR_INGEST_ERROR;
    const int64_t rows = fslr_tsv_rows(t);
    const int T = (int)std::min<int64_t>(t->n_threads, std::max<int64_t>(1, rows / 4096));
    // pass 1: per-chunk first-appearance dictionaries (local ids in local order)
    std::vector<std::unordered_map<std::string_view, int32_t>> loc((size_t)T);
    std::vector<std::vector<std::string_view>> loc_order((size_t)T);
    std::atomic<bool> ok{true}, all_int{true};
    std::vector<std::thread> pool;
    for (int c = 0; c < T; ++c)
        pool.emplace_back([&, c] {
            const int64_t a = rows * c / T, e = rows * (c + 1) / T;
            auto &m = loc[c];
            auto &ord = loc_order[c];
            bool local_int = true;
            std::string_view prev;
            int32_t prev_id = -1;
            for (int64_t i = a; i < e; ++i) {
                std::string_view f = row_field(t, i, col);
                if (is_na(f)) { ok = false; return; }
                int64_t dummy;
                if (local_int && !canon_int(f, &dummy)) local_int = false;
                int32_t id;
                if (i > a && f == prev) {
                    id = prev_id;   // rows of one read are adjacent: skip the hash lookup
                } else {
                    auto it = m.find(f);
                    if (it == m.end()) { id = (int32_t)ord.size(); m.emplace(f, id); ord.push_back(f); }
                    else id = it->second;
                }
                prev = f;
                prev_id = id;
                codes[i] = id;   // local id for now
            }
            if (!local_int) all_int = false;
        });
    for (auto &th : pool) th.join();
    pool.clear();
    if (!ok) return FSLR_INGEST_DECLINE;
    if (all_int && rows > 0) return FSLR_INGEST_DECLINE;   // pandas would type the column as int64
    // Merge, sharded by hash: shard s owns the keys with hash % T == s and walks the chunks
    // in order, so the first chunk holding a key is its global first appearance. Global ids
    // are then dense in (chunk, local order) of first appearances = pd.factorize order.
    auto run = [&](auto &&f) {
        for (int c = 0; c < T; ++c) pool.emplace_back([&, c] { f(c); });
        for (auto &th : pool) th.join();
        pool.clear();
    };
    std::vector<std::vector<uint32_t>> hs((size_t)T);
    std::vector<std::vector<int64_t>> first((size_t)T);   // -1: first appearance; else (chunk << 32 | k)
    std::vector<std::vector<int32_t>> remap((size_t)T);
    run([&](int c) {
        const auto &ord = loc_order[c];
        hs[c].resize(ord.size());
        first[c].resize(ord.size());
        remap[c].resize(ord.size());
        for (size_t k = 0; k < ord.size(); ++k) hs[c][k] = (uint32_t)(std::hash<std::string_view>{}(ord[k]) % T);
        loc[c] = {};   // local maps are no longer needed
    });
    run([&](int s) {
        std::unordered_map<std::string_view, int64_t> m;
        for (int c = 0; c < T; ++c)
            for (size_t k = 0; k < loc_order[c].size(); ++k) {
                if ((int)hs[c][k] != s) continue;
                auto r = m.try_emplace(loc_order[c][k], ((int64_t)c << 32) | (int64_t)k);
                first[c][k] = r.second ? -1 : r.first->second;
            }
    });
    std::vector<int64_t> base((size_t)T + 1, 0);
    for (int c = 0; c < T; ++c)
        base[c + 1] = base[c] + std::count(first[c].begin(), first[c].end(), (int64_t)-1);
    std::vector<std::string_view> &order = t->uniq[col];
    order.assign((size_t)base[T], std::string_view());
    run([&](int c) {
        int64_t id = base[c];
        for (size_t k = 0; k < first[c].size(); ++k)
            if (first[c][k] < 0) { remap[c][k] = (int32_t)id; order[(size_t)id++] = loc_order[c][k]; }
    });
    run([&](int c) {
        for (size_t k = 0; k < first[c].size(); ++k)
            if (first[c][k] >= 0) remap[c][k] = remap[first[c][k] >> 32][first[c][k] & 0xffffffff];
        const int64_t a = rows * c / T, e = rows * (c + 1) / T;
        const int32_t *r = remap[c].data();
        for (int64_t i = a; i < e; ++i) codes[i] = r[codes[i]];
    });
    int64_t bytes = 0;
    for (auto &s : order) bytes += (int64_t)s.size();
    *n_uniq = (int64_t)order.size();
    *uniq_bytes = bytes;
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
// Any field pandas' C parser could turn into a number.
bool numeric(std::string_view f) {
    if (f.empty()) return false;
    std::string s(f);
    char *end = nullptr;
    std::strtod(s.c_str(), &end);
    return end == s.c_str() + s.size();
}
}  // namespace

extern "C" {

int fslr_tsv_verbatim(const FslrTsv *t) {
    const int ncol = (int)t->names.size();
    const int64_t rows = fslr_tsv_rows(t);
    if (rows == 0) return FSLR_INGEST_DECLINE;
    // pandas renames empty header names ('Unnamed: N') and repeated ones ('x.1'): the input's own
    // header line would then not be what to_csv writes
    {
        std::vector<std::string> nm(t->names.begin(), t->names.end());
        for (const std::string &x : nm)
            if (x.empty()) return FSLR_INGEST_DECLINE;
        std::sort(nm.begin(), nm.end());
        if (std::adjacent_find(nm.begin(), nm.end()) != nm.end()) return FSLR_INGEST_DECLINE;
    }
    // every row exactly ncol fields: a longer row makes pandas raise (or index by the first
    // column), a shorter one NaN-fills — either way the row bytes are not what to_csv writes
    {
        std::atomic<int> ragged{0};
        const char *b = t->buf.data();
        parallel_for(rows, t->n_threads, [&](int64_t a, int64_t e, int) {
            for (int64_t i = a; i < e && !ragged.load(std::memory_order_relaxed); ++i) {
                const char *s = b + t->line[i];
                const char *le = b + t->line[rows + 1 + i];
                if (le > s && le[-1] == '\n') --le;
                if (le > s && le[-1] == '\r') --le;
                int tabs = 0;
                for (const char *q = s; (q = static_cast<const char *>(std::memchr(q, '\t', (size_t)(le - q)))) != nullptr; ++q)
                    ++tabs;
                if (tabs != ncol - 1) ragged = 1;
            }
        });
        if (ragged) return FSLR_INGEST_DECLINE;
    }
    for (int c = 0; c < ncol; ++c) {
        // 0: every field a canonical int; else the column must be text with no numeric-looking,
        // bool-looking or non-empty NA field (empty fields come back as '' either way).
        std::atomic<int> all_int{1}, text_ok{1}, any_text{0};
        parallel_for(rows, t->n_threads, [&](int64_t a, int64_t e, int) {
            bool ai = true, tk = true, at = false;
            for (int64_t i = a; i < e; ++i) {
                std::string_view f = row_field(t, i, c);
                int64_t v;
                if (ai && !canon_int(f, &v)) ai = false;
                if (!f.data()) { tk = false; continue; }   // missing field
                if (f.empty()) continue;
                if (is_na(f) || boolish(f) || numeric(f)) tk = false;
                else at = true;
            }
            if (!ai) all_int = 0;
            if (!tk) text_ok = 0;
            if (at) any_text = 1;
        });
        if (all_int) continue;
        if (!(text_ok && any_text)) return FSLR_INGEST_DECLINE;
    }
    return FSLR_INGEST_OK;
}

int fslr_tsv_write(const FslrTsv *t, const char *path, const char *header_suffix, const int64_t *rows_out,
                   int64_t n_out, const int32_t *suffix_id, const char *suffix_buf, const int64_t *suffix_ends,
                   char *err, size_t errlen) {
    FILE *fp = std::fopen(path, "wb");
    if (!fp) { set_err(err, errlen, std::string("cannot write ") + path); return FSLR_INGEST_ERROR; }
    std::string head;
    for (size_t c = 0; c < t->names.size(); ++c) { if (c) head += '\t'; head += t->names[c]; }
    head += header_suffix;
    head += '\n';
    std::fwrite(head.data(), 1, head.size(), fp);
    const int64_t rows = fslr_tsv_rows(t);
    const char *b = t->buf.data();
    const int T = std::max(1, t->n_threads);
    const int64_t block = 1 << 18;   // rows per formatting round (bounded memory)
    std::vector<std::string> part((size_t)T);
    bool bad = false;
    for (int64_t r0 = 0; r0 < n_out && !bad; r0 += block) {
        const int64_t r1 = std::min(n_out, r0 + block);
        std::atomic<bool> oob{false};
        parallel_for(r1 - r0, T, [&](int64_t a, int64_t e, int w) {
            std::string &o = part[(size_t)w];
            o.clear();
            for (int64_t k = r0 + a; k < r0 + e; ++k) {
                const int64_t i = rows_out[k];
                if (i < 0 || i >= rows) { oob = true; return; }
                const char *s = b + t->line[i];
                const char *le = b + t->line[rows + 1 + i];
                if (le > s && le[-1] == '\n') --le;
                if (le > s && le[-1] == '\r') --le;
                o.append(s, (size_t)(le - s));
                const int32_t u = suffix_id[k];
                const int64_t ss = u ? suffix_ends[u - 1] : 0;
                o.append(suffix_buf + ss, (size_t)(suffix_ends[u] - ss));
                o += '\n';
            }
        });
        if (oob) { bad = true; break; }
        const int used = (int)std::min<int64_t>(T, std::max<int64_t>(1, (r1 - r0) / 4096));
        for (int w = 0; w < used; ++w) std::fwrite(part[(size_t)w].data(), 1, part[(size_t)w].size(), fp);
    }
    if (std::fclose(fp) != 0 || bad) {
        set_err(err, errlen, bad ? "row index out of range" : "write failed");
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
  int64_t pos = 0;
  char tmp[64];
  for (int64_t k = 0; k < n_keys; ++k) {
    for (int c = 0; c < n_cols; ++c) {
      int len;
      if (kinds[c] == 0) {
        len = std::sprintf(tmp, "%lld", static_cast<long long>(static_cast<const int64_t *>(cols[c])[k]));
      } else {
        const double v = static_cast<const double *>(cols[c])[k];
        if (!std::isfinite(v)) return FSLR_INGEST_DECLINE;                // NaN / inf: pandas' own text
        len = repr_double(v, tmp);
        if (len < 0) return FSLR_INGEST_ERROR;
      }
      if (pos + len + 1 > cap) return FSLR_INGEST_ERROR;
      out[pos++] = '\t';
      std::memcpy(out + pos, tmp, static_cast<size_t>(len));
      pos += len;
    }
    ends[k] = pos;
  }
  return FSLR_INGEST_OK;
}

}  // extern "C"

// ---- CSR grouping of the prepared interval list (prepare_data order -> reads by rank) ----
extern "C" {

int fslr_group_by_first_appearance(const int64_t *codes, int64_t n, int64_t n_codes, int64_t *read_code,
                                   int64_t *n_reads, int64_t *off, int64_t *perm) {
  if (n < 0 || n_codes < 0 || (n && (!codes || !perm)) || !n_reads || !off) return FSLR_INGEST_ERROR;
  std::vector<int64_t> rank_of(static_cast<size_t>(n_codes), -1);
  int64_t nr = 0;
  for (int64_t k = 0; k < n; ++k) {                 // rank = order of first appearance (cluster.py:189-191)
    const int64_t c = codes[k];
    if (c < 0 || c >= n_codes) return FSLR_INGEST_ERROR;
    if (rank_of[c] < 0) {
      rank_of[c] = nr;
      read_code[nr] = c;
      ++nr;
    }
  }
  std::vector<int64_t> cur(static_cast<size_t>(nr) + 1, 0);
  for (int64_t k = 0; k < n; ++k) ++cur[rank_of[codes[k]] + 1];
  for (int64_t r = 0; r < nr; ++r) cur[r + 1] += cur[r];
  for (int64_t r = 0; r <= nr; ++r) off[r] = cur[r];
  for (int64_t k = 0; k < n; ++k) perm[cur[rank_of[codes[k]]]++] = k;   // stable: data order inside a read
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
