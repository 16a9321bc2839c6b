// bam.cpp — BAM record decoder for the `.mappings.bed` producer (include/fslr_bam.h).
// Host-only C++17 + zlib, built with g++ into fslr_amd/libfslr_bam.so.
//
// The file is read whole; BGZF block boundaries come from each member's BSIZE extra field
// (SAMv1 §4.1), the blocks are raw-inflated in parallel into one stream at offsets given by
// their ISIZE trailers, and the records (SAMv1 §4.2) are indexed in one sequential pass.
#include "fslr_bam.h"

#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

struct FslrBam {
  std::string data;                       // the inflated stream
  std::vector<int64_t> rec;               // offset of each record's block_size field
  std::vector<std::string> ref_name;
  std::vector<int64_t> ref_len;
  int64_t qname_bytes = 0;
};

namespace {

void set_err(char *err, size_t n, const std::string &m) {
  if (err && n) std::snprintf(err, n, "%s", m.c_str());
}

template <class T>
T rd(const char *p) {
  T v;
  std::memcpy(&v, p, sizeof(T));
  return v;
}

// BAM CIGAR op codes: M I D N S H P = X
constexpr int kOpM = 0, kOpI = 1, kOpD = 2, kOpN = 3, kOpS = 4, kOpH = 5, kOpEq = 7, kOpX = 8;

bool inflate_all(const std::string &raw, int n_threads, std::string &out, std::string &msg) {
  struct Blk { int64_t off, len, isize, dst; };
  std::vector<Blk> blocks;
  int64_t p = 0, total = 0;
  const int64_t n = static_cast<int64_t>(raw.size());
  while (p < n) {
    if (n - p < 18) { msg = "truncated BGZF block header"; return false; }
    const unsigned char *h = reinterpret_cast<const unsigned char *>(raw.data() + p);
    if (h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || !(h[3] & 4)) { msg = "not a BGZF file"; return false; }
    const int xlen = h[10] | (h[11] << 8);
    if (p + 12 + xlen > n) { msg = "truncated BGZF extra field"; return false; }
    int64_t bsize = -1;
    for (int64_t q = 12; q + 4 <= 12 + xlen;) {                 // extra subfields: find BC
      const int slen = h[q + 2] | (h[q + 3] << 8);
      if (q + 4 + slen > 12 + xlen) { msg = "BGZF extra subfield past XLEN"; return false; }
      if (h[q] == 'B' && h[q + 1] == 'C' && slen == 2) bsize = (h[q + 4] | (h[q + 5] << 8)) + 1;
      q += 4 + slen;
    }
    // the block holds its header, the extra field, the deflate data and the 8-byte CRC32 / ISIZE trailer
    if (bsize < 20 + xlen || p + bsize > n) { msg = "BGZF block without a valid BSIZE"; return false; }
    const int64_t isize = rd<uint32_t>(raw.data() + p + bsize - 4);
    if (isize > (int64_t(1) << 16)) { msg = "BGZF block with ISIZE above 64 KiB"; return false; }
    blocks.push_back({p + 12 + xlen, bsize - 12 - xlen - 8, isize, total});
    total += isize;
    p += bsize;
  }
  out.assign(static_cast<size_t>(total), '\0');
  std::atomic<int64_t> next{0};
  std::atomic<bool> ok{true};
  auto work = [&]() {
    z_stream zs;
    std::memset(&zs, 0, sizeof(zs));
    if (inflateInit2(&zs, -15) != Z_OK) { ok = false; return; }
    for (int64_t k; ok && (k = next.fetch_add(1)) < static_cast<int64_t>(blocks.size());) {
      const Blk &b = blocks[k];
      if (b.isize == 0) continue;
      inflateReset(&zs);
      zs.next_in = reinterpret_cast<Bytef *>(const_cast<char *>(raw.data() + b.off));
      zs.avail_in = static_cast<uInt>(b.len);
      zs.next_out = reinterpret_cast<Bytef *>(&out[b.dst]);
      zs.avail_out = static_cast<uInt>(b.isize);
      const int rc = inflate(&zs, Z_FINISH);
      if (rc != Z_STREAM_END || zs.avail_out != 0) ok = false;
    }
    inflateEnd(&zs);
  };
  int t = n_threads > 0 ? n_threads : static_cast<int>(std::thread::hardware_concurrency());
  t = std::max(1, std::min<int>(t, static_cast<int>(std::min<size_t>(blocks.size(), 64))));
  std::vector<std::thread> pool;
  for (int k = 1; k < t; ++k) pool.emplace_back(work);
  work();
  for (auto &th : pool) th.join();
  if (!ok) { msg = "corrupt BGZF block"; return false; }
  return true;
}

}  // namespace

extern "C" {

int fslr_bam_open(const char *path, int n_threads, FslrBam **out, char *err, size_t errlen) {
  if (!path || !out) return FSLR_BAM_ERROR;
  *out = nullptr;
  FILE *f = std::fopen(path, "rb");
  if (!f) { set_err(err, errlen, std::string("cannot open ") + path); return FSLR_BAM_ERROR; }
  std::string raw;
  std::fseek(f, 0, SEEK_END);
  const long sz = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  raw.resize(static_cast<size_t>(sz > 0 ? sz : 0));
  const size_t got = sz > 0 ? std::fread(&raw[0], 1, raw.size(), f) : 0;
  std::fclose(f);
  if (got != raw.size()) { set_err(err, errlen, "short read"); return FSLR_BAM_ERROR; }
  auto *b = new FslrBam();
  std::string msg;
  if (!inflate_all(raw, n_threads, b->data, msg)) {
    set_err(err, errlen, msg);
    delete b;
    return FSLR_BAM_ERROR;
  }
  raw.clear();
  raw.shrink_to_fit();
  const std::string &d = b->data;
  const int64_t n = static_cast<int64_t>(d.size());
  auto fail = [&](const char *m) {
    set_err(err, errlen, m);
    delete b;
    return FSLR_BAM_ERROR;
  };
  if (n < 12 || std::memcmp(d.data(), "BAM\1", 4) != 0) return fail("not a BAM file (bad magic)");
  int64_t p = 4;
  const int32_t l_text = rd<int32_t>(d.data() + p);
  p += 4 + l_text;
  if (l_text < 0 || p + 4 > n) return fail("truncated BAM header");
  const int32_t n_ref = rd<int32_t>(d.data() + p);
  p += 4;
  for (int k = 0; k < n_ref; ++k) {
    if (p + 4 > n) return fail("truncated reference list");
    const int32_t l_name = rd<int32_t>(d.data() + p);
    if (l_name < 1 || p + 8 + l_name > n) return fail("truncated reference list");
    b->ref_name.emplace_back(d.data() + p + 4, static_cast<size_t>(l_name - 1));
    b->ref_len.push_back(rd<int32_t>(d.data() + p + 4 + l_name));
    p += 8 + l_name;
  }
  while (p < n) {
    if (p + 36 > n) return fail("truncated alignment record");
    const int32_t bs = rd<int32_t>(d.data() + p);
    if (bs < 32 || p + 4 + bs > n) return fail("bad alignment record size");
    const int l_name = static_cast<unsigned char>(d[p + 12]);
    const int64_t nc = rd<uint16_t>(d.data() + p + 16);
    const int64_t ls = rd<int32_t>(d.data() + p + 20);
    // the fixed fields, read name, CIGAR, packed sequence and qualities lie inside the record
    if (l_name < 1 || ls < 0 || 36 + l_name + 4 * nc + (ls + 1) / 2 + ls > 4 + static_cast<int64_t>(bs))
      return fail("alignment record fields past its end");
    b->qname_bytes += std::max(0, l_name - 1);
    b->rec.push_back(p);
    p += 4 + bs;
  }
  *out = b;
  return FSLR_BAM_OK;
}

void fslr_bam_close(FslrBam *b) { delete b; }

int64_t fslr_bam_n_records(const FslrBam *b) { return b ? static_cast<int64_t>(b->rec.size()) : -1; }
int fslr_bam_n_refs(const FslrBam *b) { return b ? static_cast<int>(b->ref_name.size()) : -1; }
const char *fslr_bam_ref_name(const FslrBam *b, int tid) {
  return b && tid >= 0 && tid < static_cast<int>(b->ref_name.size()) ? b->ref_name[tid].c_str() : nullptr;
}
int64_t fslr_bam_ref_len(const FslrBam *b, int tid) {
  return b && tid >= 0 && tid < static_cast<int>(b->ref_len.size()) ? b->ref_len[tid] : -1;
}
int64_t fslr_bam_qname_bytes(const FslrBam *b) { return b ? b->qname_bytes : -1; }

int fslr_bam_columns(const FslrBam *b, int32_t *flag, int32_t *tid, int64_t *pos, int32_t *mapq, int64_t *ref_span,
                     int64_t *read_len, int64_t *clip_first, int64_t *clip_last, int32_t *n_cigar, int64_t *as_tag,
                     int8_t *as_kind, int64_t *l_seq, int64_t *qname_end, char *qname_buf) {
  if (!b) return FSLR_BAM_ERROR;
  int64_t qn = 0;
  const char *base = b->data.data();
  for (size_t k = 0; k < b->rec.size(); ++k) {
    const char *r = base + b->rec[k];
    const char *end = r + 4 + rd<int32_t>(r);
    tid[k] = rd<int32_t>(r + 4);
    pos[k] = rd<int32_t>(r + 8);
    const int l_name = static_cast<unsigned char>(r[12]);
    mapq[k] = static_cast<unsigned char>(r[13]);
    const int nc = rd<uint16_t>(r + 16);
    flag[k] = rd<uint16_t>(r + 18);
    const int32_t ls = rd<int32_t>(r + 20);
    l_seq[k] = ls;
    n_cigar[k] = nc;
    const char *name = r + 36;
    const int nlen = std::max(0, l_name - 1);
    std::memcpy(qname_buf + qn, name, static_cast<size_t>(nlen));
    qn += nlen;
    qname_end[k] = qn;
    const char *cg = name + l_name;
    int64_t span = 0, rlen = 0;
    clip_first[k] = clip_last[k] = 0;
    for (int c = 0; c < nc; ++c) {
      const uint32_t v = rd<uint32_t>(cg + 4 * c);
      const int op = v & 15;
      const int64_t len = v >> 4;
      if (op == kOpM || op == kOpD || op == kOpN || op == kOpEq || op == kOpX) span += len;
      if (op == kOpM || op == kOpI || op == kOpS || op == kOpEq || op == kOpX || op == kOpH) rlen += len;
      if ((op == kOpS || op == kOpH) && c == 0) clip_first[k] = len;
      if ((op == kOpS || op == kOpH) && c == nc - 1) clip_last[k] = len;
    }
    ref_span[k] = span;
    read_len[k] = rlen;
    // tags after seq and qual
    const char *t = cg + 4 * nc + (ls + 1) / 2 + ls;
    as_kind[k] = 0;
    as_tag[k] = 0;
    while (t + 3 <= end) {
      const char t0 = t[0], t1 = t[1], ty = t[2];
      const char *v = t + 3;
      const int64_t room = end - v;
      int64_t ival = 0;
      int isint = 1, size = 0;
      switch (ty) {
        case 'A': size = 1; isint = 0; break;
        case 'c': if (room < 1) return FSLR_BAM_ERROR; ival = rd<int8_t>(v); size = 1; break;
        case 'C': if (room < 1) return FSLR_BAM_ERROR; ival = rd<uint8_t>(v); size = 1; break;
        case 's': if (room < 2) return FSLR_BAM_ERROR; ival = rd<int16_t>(v); size = 2; break;
        case 'S': if (room < 2) return FSLR_BAM_ERROR; ival = rd<uint16_t>(v); size = 2; break;
        case 'i': if (room < 4) return FSLR_BAM_ERROR; ival = rd<int32_t>(v); size = 4; break;
        case 'I': if (room < 4) return FSLR_BAM_ERROR; ival = rd<uint32_t>(v); size = 4; break;
        case 'f': size = 4; isint = 0; break;
        case 'Z': case 'H': {
          if (room <= 0) return FSLR_BAM_ERROR;
          const void *z = std::memchr(v, 0, static_cast<size_t>(room));
          if (!z) return FSLR_BAM_ERROR;
          size = static_cast<int>(static_cast<const char *>(z) - v) + 1;
          isint = 0;
          break;
        }
        case 'B': {
          if (room < 5) return FSLR_BAM_ERROR;
          const char sub = v[0];
          const int32_t cnt = rd<int32_t>(v + 1);
          const int es = (sub == 'c' || sub == 'C') ? 1 : (sub == 's' || sub == 'S') ? 2
                       : (sub == 'i' || sub == 'I' || sub == 'f') ? 4 : 0;
          if (!es || cnt < 0 || 5 + static_cast<int64_t>(es) * cnt > room) return FSLR_BAM_ERROR;
          size = 5 + es * cnt;
          isint = 0;
          break;
        }
        default: return FSLR_BAM_ERROR;
      }
      if (size > room) return FSLR_BAM_ERROR;         // a fixed-size value cut off by the record end
      if (t0 == 'A' && t1 == 'S' && as_kind[k] == 0) {
        as_kind[k] = isint ? 1 : 2;
        as_tag[k] = ival;
      }
      t = v + size;
    }
  }
  return FSLR_BAM_OK;
}

int fslr_bam_forward_seq(const FslrBam *b, int64_t rec, char *out) {
  if (!b || rec < 0 || rec >= static_cast<int64_t>(b->rec.size())) return FSLR_BAM_ERROR;
  static const char kCode[] = "=ACMGRSVTWYHKDBN";
  const char *r = b->data.data() + b->rec[rec];
  const int l_name = static_cast<unsigned char>(r[12]);
  const int nc = rd<uint16_t>(r + 16);
  const int flag = rd<uint16_t>(r + 18);
  const int32_t ls = rd<int32_t>(r + 20);
  const unsigned char *s = reinterpret_cast<const unsigned char *>(r + 36 + l_name + 4 * nc);
  for (int32_t i = 0; i < ls; ++i) out[i] = kCode[(s[i >> 1] >> ((~i & 1) << 2)) & 15];
  if (flag & 16) {
    std::reverse(out, out + ls);
    for (int32_t i = 0; i < ls; ++i) {
      char &c = out[i];
      c = c == 'A' ? 'T' : c == 'T' ? 'A' : c == 'C' ? 'G' : c == 'G' ? 'C' : c;
    }
  }
  return FSLR_BAM_OK;
}

}  // extern "C"
