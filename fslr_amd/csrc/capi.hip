// capi.hip — the C ABI (include/fslr_hip.h): context, HBM buffers, launch sequencing, timing.
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "fslr_hip.h"
#include "ctx.hpp"
#include "kernels.hpp"

using namespace fslr;

namespace {

int alloc_errw(fslr_ctx* c, int cap);

int ensure_capacity(fslr_ctx* c, int64_t n, int64_t ni, int n_chroms) {
  int rc;
  if (n > c->cap_n) {
    if ((rc = dalloc(c, &c->rmeta, n)) || (rc = dalloc(c, &c->rlen8, n)) || (rc = dalloc(c, &c->fwd, n)) ||
        (rc = dalloc(c, &c->parent, n)) || (rc = dalloc(c, &c->forest, n)) ||
        (rc = dalloc(c, &c->heavy, n)) ||
        (rc = dalloc(c, &c->lbounds, n)))
      return rc;
#ifdef FSLR_SECTION_PROF
    if ((rc = dalloc(c, &c->diag, 2 * n))) return rc;
#endif
    c->cap_n = n;
  }
  if (ni > c->cap_ni) {
    if ((rc = dalloc(c, &c->iv, ni)) || (rc = dalloc(c, &c->qpos, ni)) || (rc = dalloc(c, &c->rng_s, ni)) || (rc = dalloc(c, &c->swin, ni)) || (rc = dalloc(c, &c->idx4, ni)) ||
        (rc = dalloc(c, &c->idx_gate, ni)) || (rc = dalloc(c, &c->data_pos, ni)) ||
        (rc = dalloc(c, &c->dchrom, ni)) || (rc = dalloc(c, &c->drec, ni)) || (rc = dalloc(c, &c->dgate, ni)) ||
        (rc = dalloc(c, &c->chist, (ni / 1024 + 1) * 64)) || (rc = dalloc(c, &c->s_start, ni)) ||
        (rc = dalloc(c, &c->keys, ni)) || (rc = dalloc(c, &c->keys2, ni)) || (rc = dalloc(c, &c->vals, ni)) ||
        (rc = dalloc(c, &c->vals2, ni)) || (rc = dalloc(c, &c->endkey, ni)) || (rc = dalloc(c, &c->pmaxkey, 2 * (ni / 256) + ni / (256 * 1024) + 8)) ||
        (rc = dalloc(c, &c->thr_tmp, ni)))
      return rc;
    c->cap_ni = ni;
    size_t need = 0;
    HIP_TRY(c, index_temp_bytes(static_cast<int>(ni), &need, c->stream));
    if (need > c->temp_bytes) {
      if (c->temp) (void)hipFree(c->temp);
      c->temp = nullptr;
      HIP_TRY(c, hipMalloc(&c->temp, need));
      c->temp_bytes = need;
    }
  }
  if (n_chroms > c->cap_chroms) {
    if ((rc = dalloc(c, &c->crange, n_chroms))) return rc;
    c->cap_chroms = n_chroms;
  }
  if (!c->umax) {
    if ((rc = dalloc(c, &c->umax, FSLR_MAX_L))) return rc;
    if ((rc = dalloc(c, &c->counters, kNumCounters))) return rc;
    if ((rc = alloc_errw(c, kZdListInit))) return rc;
    if ((rc = dalloc(c, &c->forest_cnt, 1))) return rc;
    if ((rc = dalloc(c, &c->forest_blk, 1024))) return rc;
    // no query yet: no edges, no errors (fslr_components before any query gives singleton labels)
    HIP_TRY(c, hipMemsetAsync(c->counters, 0, kNumCounters * sizeof(unsigned long long), c->stream));
  }
  return FSLR_OK;
}

// the error words and the ZeroDivisionError pair list after them (kernels.hpp kErrZdList), zeroed, with
// the list's capacity in word kErrZdCap
int alloc_errw(fslr_ctx* c, int cap) {
  if (int rc = dalloc(c, &c->errw, kErrZdList + 2 * static_cast<size_t>(cap))) return rc;
  c->zd_cap = cap;
  HIP_TRY(c, hipMemsetAsync(c->errw, 0, kErrZdList * sizeof(int), c->stream));
  HIP_TRY(c, hipMemcpyAsync(c->errw + kErrZdCap, &c->zd_cap, sizeof(int), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FSLR_OK;
}

// the sweep's match-entry buffers and their grouping-sort scratch (grow only)
int reserve_entries(fslr_ctx* c, int64_t capacity) {
  if (capacity <= c->ent_cap) return FSLR_OK;
  if (capacity >= (int64_t(1) << 31)) return fail(c, FSLR_ERR_NOMEM, "more than 2^31 match entries");
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  int rc;
  if ((rc = dalloc(c, &c->ent, capacity)) || (rc = dalloc(c, &c->ent_sorted, capacity))) return rc;
  const size_t need = sweep_temp_bytes(capacity, std::max<int64_t>(std::max(c->ni, c->n), 64), c->stream);
  if (need > c->sweep_temp_bytes) {
    if (c->sweep_temp) (void)hipFree(c->sweep_temp);
    c->sweep_temp = nullptr;
    HIP_TRY(c, hipMalloc(&c->sweep_temp, need));
    c->sweep_temp_bytes = need;
  }
  c->ent_cap = capacity;
  return FSLR_OK;
}

// the grouping sort's bucket counts and offsets (fixed size)
static int ensure_grp(fslr_ctx* c) {
  if (c->grp) return FSLR_OK;
  return dalloc(c, &c->grp, grp_ints());
}

// f(a, e, w) over [0, n) in contiguous slices on up to 16 host threads ($OMP_NUM_THREADS); the input
// packing of fslr_set_reads touches every interval a few times (62M at cfg5)
int host_threads(int64_t n) {
  const char* env = std::getenv("OMP_NUM_THREADS");
  int t = env ? std::atoi(env) : 0;
  if (t <= 0) t = static_cast<int>(std::min(16u, std::max(1u, std::thread::hardware_concurrency())));
  return static_cast<int>(std::min<int64_t>(std::min(t, 256), std::max<int64_t>(1, n / 65536)));
}

template <class F>
void host_for(int64_t n, F f) {
  const int t = host_threads(n);
  if (t <= 1) {
    f(int64_t(0), n, 0);
    return;
  }
  std::vector<std::thread> pool;
  for (int i = 0; i < t; ++i) pool.emplace_back([=, &f] { f(n * i / t, n * (i + 1) / t, i); });
  for (auto& th : pool) th.join();
}

int thr_mode_of(const int32_t* thr, int64_t ni) {
  for (int64_t k = 0; k < ni; ++k)
    if (thr[k] != FSLR_THR_ZERO_ALN && thr[k] < 1) return 1;
  return 0;
}

}  // namespace

extern "C" {

int fslr_abi_version(void) { return FSLR_ABI_VERSION; }

const char* fslr_last_error(const fslr_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int fslr_ctx_create(int device, void* stream, fslr_ctx** out) {
  if (!out) return FSLR_ERR_INVALID;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return FSLR_ERR_HIP;
  if (device < 0 || device >= ndev) return FSLR_ERR_INVALID;
  if (hipSetDevice(device) != hipSuccess) return FSLR_ERR_HIP;
  fslr_ctx* c = new fslr_ctx();
  c->device = device;
  if (stream) {
    c->stream = static_cast<hipStream_t>(stream);
  } else {
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
      delete c;
      return FSLR_ERR_HIP;
    }
    c->own_stream = true;
  }
  if (const char* m = std::getenv("FSLR_ABLATE")) c->ablate = std::atoi(m);   // profiling only
  *out = c;
  return FSLR_OK;
}

void fslr_ctx_destroy(fslr_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  void* bufs[] = {c->rmeta,  c->rlen8, c->iv,     c->qpos,    c->rng_s,  c->swin, c->idx4,    c->idx_gate, c->data_pos, c->s_start,
                  c->crange, c->keys,   c->keys2,   c->vals,    c->vals2,   c->endkey,  c->pmaxkey,
                  c->temp,   c->umax,   c->edges,   c->edge_iu, c->fwd,     c->parent,  c->counters, c->forest, c->forest_cnt, c->forest_blk,
                  c->upl,    c->upl64,
                  c->errw,   c->thr_tmp, c->defer,   c->dchrom,  c->drec,    c->lbounds, c->diag, c->wstat,
                  c->dgate,  c->chist,  c->heavy, c->ent, c->ent_sorted, c->sweep_temp, c->sw_tile, c->sw_wstat, c->sw_wlo, c->ent_ub,
                  c->fdchrom, c->fdrec, c->fdgate, c->crange_f, c->part_cnt, c->grp, c->fmap,
                  c->rows_col, c->rows_ord, c->rows_keep, c->rows_int, c->rows_l, c->rows_temp,
                  c->pf_sel, c->pf_lmap, c->pf_cost};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  if (c->sw_total) (void)hipHostFree(c->sw_total);
  fslr_long_free(c);
  fslr_cap_free(c);
  if (c->ev_ok) {
    for (auto& e : c->ev) (void)hipEventDestroy(e);
    for (auto& e : c->kev) (void)hipEventDestroy(e);
    for (auto& e : c->kev2) (void)hipEventDestroy(e);
    for (auto& e : c->sw_ev) (void)hipEventDestroy(e);
  }
  if (c->own_stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int fslr_set_query_reuse(fslr_ctx* c, int enable) {
  if (!c) return FSLR_ERR_INVALID;
  c->reuse = enable != 0;
  return FSLR_OK;
}

int fslr_set_profiling(fslr_ctx* c, int enable) {
  if (!c) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  if (enable && !c->ev_ok) {
    // timing-only events: no system-scope fence at record (its cache writeback and invalidation
    // would cost every profiled step a bubble and start the next kernel on cold caches)
    const unsigned fl = hipEventDisableSystemFence;
    for (auto& e : c->ev) HIP_TRY(c, hipEventCreateWithFlags(&e, fl));
    c->kev.assign(2 * fslr_ctx::kKernRing, nullptr);
    for (auto& e : c->kev) HIP_TRY(c, hipEventCreateWithFlags(&e, fl));
    c->kev2.assign(2 * fslr_ctx::kKernRing, nullptr);
    for (auto& e : c->kev2) HIP_TRY(c, hipEventCreateWithFlags(&e, fl));
    for (auto& e : c->sw_ev) HIP_TRY(c, hipEventCreateWithFlags(&e, fl));
    c->ev_ok = true;
  }
  c->profiling = enable != 0;
  c->prof_phases = enable == 1;
  return FSLR_OK;
}

int fslr_set_reads(fslr_ctx* c, const fslr_reads* r) {
  if (!c || !r) return FSLR_ERR_INVALID;
  c->hooked = false;
  HIP_TRY(c, hipSetDevice(c->device));
  const int64_t n = r->n_reads, ni = r->n_intervals;
  if (n < 0 || ni < 0 || n >= FSLR_MAX_READS || ni >= (int64_t(1) << 31) - 1)
    return fail(c, FSLR_ERR_INVALID, "read / interval count out of range");
  if (r->n_chroms < 1 || r->n_chroms >= (1 << 24)) return fail(c, FSLR_ERR_INVALID, "n_chroms out of range");
  if (!r->read_off || !r->read_qlen2 || !r->read_nal || !r->iv_chrom || !r->iv_start || !r->iv_end || !r->iv_thr)
    return fail(c, FSLR_ERR_INVALID, "null array");
  if (r->read_off[0] != 0 || r->read_off[n] != ni)
    return fail(c, FSLR_ERR_INVALID, "read_off does not span intervals");
  hipStream_t st = c->stream;
  int rc = ensure_capacity(c, n, ni, r->n_chroms);
  if (rc) return rc;
  const int64_t upl_need = 3 * n + 1 + 4 * ni;
  if (upl_need > c->upl_cap) {
    if ((rc = dalloc(c, &c->upl, static_cast<size_t>(upl_need)))) return rc;
    c->upl_cap = upl_need;
  }
  if (r->n_chroms + 2 > c->upl64_cap) {
    if ((rc = dalloc(c, &c->upl64, static_cast<size_t>(r->n_chroms + 2)))) return rc;
    c->upl64_cap = r->n_chroms + 2;
  }
  // the caller's columns to the device as they are; validation and packing run there (upload.hip)
  int* d_off = c->upl;
  int* d_q2 = d_off + n + 1;
  int* d_nal = d_q2 + n;
  int* d_ch = d_nal + n;
  int* d_st = d_ch + ni;
  int* d_en = d_st + ni;
  int* d_th = d_en + ni;
  unsigned long long* d_cnt = c->upl64;
  unsigned long long* d_err = c->upl64 + r->n_chroms;
  const size_t nb = static_cast<size_t>(n) * sizeof(int), ib = static_cast<size_t>(ni) * sizeof(int);
  HIP_TRY(c, hipMemsetAsync(d_cnt, 0, static_cast<size_t>(r->n_chroms) * sizeof(unsigned long long), st));
  HIP_TRY(c, hipMemsetAsync(d_err, 0xff, 2 * sizeof(unsigned long long), st));
  HIP_TRY(c, hipMemcpyAsync(d_off, r->read_off, nb + sizeof(int), hipMemcpyHostToDevice, st));
  if (n) {
    HIP_TRY(c, hipMemcpyAsync(d_q2, r->read_qlen2, nb, hipMemcpyHostToDevice, st));
    HIP_TRY(c, hipMemcpyAsync(d_nal, r->read_nal, nb, hipMemcpyHostToDevice, st));
  }
  if (ni) {
    HIP_TRY(c, hipMemcpyAsync(d_ch, r->iv_chrom, ib, hipMemcpyHostToDevice, st));
    HIP_TRY(c, hipMemcpyAsync(d_st, r->iv_start, ib, hipMemcpyHostToDevice, st));
    HIP_TRY(c, hipMemcpyAsync(d_en, r->iv_end, ib, hipMemcpyHostToDevice, st));
    HIP_TRY(c, hipMemcpyAsync(d_th, r->iv_thr, ib, hipMemcpyHostToDevice, st));
    if (r->iv_data_pos) HIP_TRY(c, hipMemcpyAsync(c->data_pos, r->iv_data_pos, ib, hipMemcpyHostToDevice, st));
  }
  // the reads' own checks on the host (a read's intervals must lie in [0, ni) before the device reads
  // them); per slice the code of its first failure: 3 read length, 4 n_alignments, 5 qlen2 — slices are
  // contiguous in index order, so the lowest failing slice holds the input's first failure
  std::vector<int> bad_slice(static_cast<size_t>(std::max(host_threads(ni), host_threads(n))), 0);
  host_for(n, [&](int64_t a, int64_t e, int w) {
    for (int64_t i = a; i < e; ++i) {
      const int len = r->read_off[i + 1] - r->read_off[i];
      if (len < 1 || len > FSLR_MAX_L) { bad_slice[w] = 3; return; }
      if (r->read_nal[i] < 0 || r->read_nal[i] >= (1 << 24)) { bad_slice[w] = 4; return; }
      if (r->read_qlen2[i] < 0) { bad_slice[w] = 5; return; }   // max(qend) - min(qstart) over a read's fillings (cluster.py:26-29)
    }
  });
  int bad = 0;
  for (int b : bad_slice)
    if (b) { bad = b; break; }
  UploadArgs ua{};
  ua.off = d_off;
  ua.qlen2 = d_q2;
  ua.nal = d_nal;
  ua.chrom = d_ch;
  ua.start = d_st;
  ua.end = d_en;
  ua.thr = d_th;
  ua.dp = r->iv_data_pos ? c->data_pos : nullptr;
  ua.n = static_cast<int>(n);
  ua.ni = static_cast<int>(ni);
  ua.n_chroms = r->n_chroms;
  ua.reads_ok = bad == 0;
  ua.iv = c->iv;
  ua.rmeta = c->rmeta;
  ua.rlen8 = c->rlen8;
  ua.dch = c->dchrom;
  ua.drc = c->drec;
  ua.dgt = c->dgate;
  ua.inv = c->vals2;
  ua.chrom_cnt = d_cnt;
  ua.err = d_err;
  HIP_TRY(c, launch_upload_pack(ua, st));
  // beside the device: the aln_size == 0 marks (fslr_set_thresholds checks them) and the threshold mode
  std::vector<unsigned char> zero(static_cast<size_t>(ni), 0);
  std::vector<int> any_zero(static_cast<size_t>(host_threads(ni)), 0);
  host_for(ni, [&](int64_t a, int64_t e, int w) {
    int z = 0;
    for (int64_t k = a; k < e; ++k) {
      const unsigned char f = r->iv_thr[k] == FSLR_THR_ZERO_ALN;
      zero[k] = f;
      z |= f;
    }
    any_zero[w] = z;
  });
  const int tmode = thr_mode_of(r->iv_thr, ni);
  std::vector<int64_t> chrom_counts(static_cast<size_t>(r->n_chroms), 0);
  unsigned long long err[2] = {0, 0};
  HIP_TRY(c, hipMemcpyAsync(chrom_counts.data(), d_cnt, chrom_counts.size() * sizeof(int64_t), hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipMemcpyAsync(err, d_err, sizeof(err), hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipStreamSynchronize(st));
  c->reads_set = false;
  if (err[0] != ~0ull) {
    if ((err[0] & 7) == kUpErrChrom) return fail(c, FSLR_ERR_INVALID, "chrom id out of range");
    return fail(c, FSLR_ERR_INVALID, "interval coordinates out of [0, 2^30)");
  }
  if (bad == 3) return fail(c, FSLR_ERR_INVALID, "every read needs 1.." + std::to_string(FSLR_MAX_L) + " intervals");
  if (bad == 4) return fail(c, FSLR_ERR_INVALID, "n_alignments outside [0, 2^24)");
  if (bad == 5) return fail(c, FSLR_ERR_INVALID, "qlen2 < 0");
  if (err[1] != ~0ull) return fail(c, FSLR_ERR_INVALID, "iv_data_pos is not a start-sorted permutation");
  // chromosome ranges of the (chrom, start)-sorted index: chromosome ids ascending
  std::vector<int2> cr(static_cast<size_t>(r->n_chroms), make_int2(0, 0));
  int64_t acc = 0;
  for (int ch = 0; ch < r->n_chroms; ++ch) {
    cr[ch] = make_int2(static_cast<int>(acc), static_cast<int>(acc + chrom_counts[ch]));
    acc += chrom_counts[ch];
  }
  HIP_TRY(c, hipMemcpyAsync(c->crange, cr.data(), cr.size() * sizeof(int2), hipMemcpyHostToDevice, st));
  HIP_TRY(c, hipStreamSynchronize(st));
  c->have_data_pos = r->iv_data_pos != nullptr;
  c->rows_set = false;
  c->n = n;
  c->ni = ni;
  c->ni_idx = ni;
  c->filter_active = false;
  c->chrom_counts.swap(chrom_counts);
  c->n_chroms = r->n_chroms;
  c->thr_mode = tmode;
  c->any_zero_aln = std::find(any_zero.begin(), any_zero.end(), 1) != any_zero.end();
  c->aln_zero_host.swap(zero);
  c->reads_set = true;
  ++c->reads_gen;
  c->pf_set = c->pf_on = false;
  c->index_built = false;
  c->lg_set = false;                        // a virtual-read map belongs to the reads it was set for
  c->lg_perm.clear();
  c->edges_global = false;
  c->cap_gmode = false;
  ++c->input_gen;
  return FSLR_OK;
}

static IndexBufs index_bufs(fslr_ctx* c);

// thr_tmp (the new folded thresholds, CSR order) into every copy of them: iv, the data-order records, the
// sorted index, the sweep windows (start_p <= end_q - thr_q decides swin) and the filtered records of a
// chromosome or position filter. ensure_walk_index(c) first: idx4 is updated through qpos.
static int install_thresholds(fslr_ctx* c) {
  HIP_TRY(c, launch_set_thr(c->thr_tmp, c->iv, c->qpos, c->index_built ? c->idx4 : nullptr, c->data_pos,
                            c->have_data_pos ? c->drec : nullptr, static_cast<int>(c->ni), c->stream));
  if (c->index_built) {
    const IndexBufs b = index_bufs(c);
    HIP_TRY(c, launch_index_swin(b, static_cast<int>(c->ni_idx), c->stream));
  }
  c->idx_tt_valid = false;                        // the windows changed: the plan sums them again
  if (c->filter_active && c->pf_on)
    HIP_TRY(c, launch_pos_gather(c->pf_sel, static_cast<int>(c->pf_end - c->pf_lo), c->dchrom, c->drec, c->dgate,
                                 c->pf_lmap, c->fdchrom, c->fdrec, c->fdgate, c->stream));
  else if (c->filter_active)
    HIP_TRY(c, launch_chrom_filter(c->dchrom, c->drec, c->dgate, c->fmap, static_cast<int>(c->ni), c->fdchrom,
                                   c->fdrec, c->fdgate, c->vals2, c->vals, c->temp, c->temp_bytes, c->stream));
  ++c->thr_gen;                  // a position plan's halo was cut for the windows of the old thresholds
  return FSLR_OK;
}

int fslr_set_thresholds(fslr_ctx* c, const int32_t* thr_in) {
  if (!c || (!thr_in && c->ni)) return FSLR_ERR_INVALID;
  if (!c->reads_set) return fail(c, FSLR_ERR_STATE, "fslr_set_reads first");
  ++c->input_gen;
  // reads uploaded by fslr_set_reads_any: the thresholds come in the real CSR's interval order
  std::vector<int32_t> permuted;
  const int32_t* thr = thr_in;
  if (!c->lg_perm.empty()) {
    permuted.resize(c->lg_perm.size());
    for (size_t k = 0; k < permuted.size(); ++k) permuted[k] = thr_in[c->lg_perm[k]];
    thr = permuted.data();
  }
  HIP_TRY(c, hipSetDevice(c->device));
  for (int64_t k = 0; k < c->ni; ++k)
    if ((thr[k] == FSLR_THR_ZERO_ALN) != (c->aln_zero_host[k] != 0))
      return fail(c, FSLR_ERR_INVALID, "FSLR_THR_ZERO_ALN must mark the same intervals as in fslr_set_reads");
  if (c->ni) {
    HIP_TRY(c, hipMemcpyAsync(c->thr_tmp, thr, c->ni * sizeof(int), hipMemcpyHostToDevice, c->stream));
    if (c->index_built && (c->built_n_shards != 1 || c->filter_active))
      c->index_built = false;                                               // qpos is partial: rebuild
    int rc = ensure_walk_index(c);                                           // idx4 is updated through qpos
    if (rc) return rc;
    if (int rc = install_thresholds(c)) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
  }
  c->thr_mode = thr_mode_of(thr, c->ni);
  return FSLR_OK;
}

// ---- the clustering input from rows (rows.hip) ------------------------------------------------------
int fslr_rows_upload(fslr_ctx* c, const fslr_rows* r) {
  if (!c || !r || r->n_rows < 1 || r->n_rows >= (int64_t(1) << 31) - 1 || r->n_codes < 1 ||
      r->n_codes >= (int64_t(1) << 31) || r->n_chrom_ids < 1 || r->n_chrom_ids >= (1 << 24))
    return FSLR_ERR_INVALID;
  c->hooked = false;
  if (!r->chrom || !r->start || !r->end || !r->aln || !r->qcode || !r->nal || !r->qlen2)
    return fail(c, FSLR_ERR_INVALID, "null array");
  HIP_TRY(c, hipSetDevice(c->device));
  const int64_t n = r->n_rows;
  c->rows_n = 0;
  // the device-made CSR's views (fslr_get_csr, fslr_get_read_codes, fslr_fold_thresholds) are laid out
  // over rows_cap and the old code / chromosome counts: they end here, and with them the reads they made
  if (c->rows_set) {
    c->rows_set = false;
    c->reads_set = false;
    c->index_built = false;
    ++c->input_gen;
  }
  if (n > c->rows_cap) {
    int rc;
    if ((rc = dalloc(c, &c->rows_col, 7 * static_cast<size_t>(n))) || (rc = dalloc(c, &c->rows_ord, n)) ||
        (rc = dalloc(c, &c->rows_keep, n)) || (rc = dalloc(c, &c->rows_l, 2 * static_cast<size_t>(n))))
      return rc;
    c->rows_cap = n;
  }
  const int64_t* src[7] = {r->chrom, r->start, r->end, r->aln, r->qcode, r->nal, r->qlen2};
  for (int k = 0; k < 7; ++k)
    HIP_TRY(c, hipMemcpyAsync(c->rows_col + k * n, src[k], static_cast<size_t>(n) * sizeof(long long),
                              hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->rows_n = n;
  c->rows_codes = r->n_codes;
  c->rows_cids = r->n_chrom_ids;
  return FSLR_OK;
}

namespace {
// the build's views of the rows arenas (capacity rows_cap; the per-code and per-chromosome arrays last)
RowsWork rows_views(fslr_ctx* c) {
  const int64_t n = c->rows_cap;
  RowsWork w{};
  const long long* col = c->rows_col;
  w.chrom = col;
  w.start = col + n;
  w.end = col + 2 * n;
  w.aln = col + 3 * n;
  w.qcode = col + 4 * n;
  w.nal = col + 5 * n;
  w.qlen2 = col + 6 * n;
  int* p = c->rows_int;
  auto take = [&](int64_t k) {
    int* q = p;
    p += (k + 63) / 64 * 64;
    return q;
  };
  w.ord32 = take(n);
  w.flag = reinterpret_cast<unsigned char*>(take(n / 4 + 1));
  w.sel = take(n);
  w.nsel = take(1);
  w.f = take(n);
  w.fscan = take(n);
  w.key = take(n);
  w.val = take(n);
  w.key_s = take(n);
  w.perm = take(n);
  w.off = take(n + 1);
  w.ch_raw = take(n);
  w.st32 = take(n);
  w.en32 = take(n);
  w.dp = take(n);            // the index build reads the data order from c->data_pos (a copy below)
  w.q2 = take(n);
  w.nal32 = take(n);
  w.present = take(c->rows_cids);
  w.stat = take(4);
  w.err = take(1);
  w.first = take(c->rows_codes);
  w.aln_k = c->rows_l;
  w.code_of_rank = c->rows_l + n;
  w.temp = c->rows_temp;
  w.temp_bytes = c->rows_temp_bytes;
  return w;
}

int64_t rows_int_need(int64_t n, int64_t codes, int64_t cids) {
  return 20 * ((n + 64) / 64 * 64 + 64) + (codes + 63) / 64 * 64 + (cids + 63) / 64 * 64 + 4 * 64 + 4 * n;
}
}  // namespace

int fslr_set_reads_rows(fslr_ctx* c, const int64_t* order, const uint8_t* keep, double overlap,
                        fslr_rows_info* info) {
  if (!c || !order || !info) return FSLR_ERR_INVALID;
  c->hooked = false;
  std::memset(info, 0, sizeof(*info));
  const int64_t n = c->rows_n;
  if (n < 1) return fail(c, FSLR_ERR_STATE, "fslr_rows_upload first");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t st = c->stream;
  int rc;
  const int64_t need = rows_int_need(c->rows_cap, c->rows_codes, c->rows_cids) + 2 * c->rows_cids;
  if (need > c->rows_int_cap) {
    if ((rc = dalloc(c, &c->rows_int, static_cast<size_t>(need)))) return rc;
    c->rows_int_cap = need;
  }
  const size_t tb = rows_temp_bytes(c->rows_cap, st);
  if (tb > c->rows_temp_bytes) {
    if (c->rows_temp) (void)hipFree(c->rows_temp);
    c->rows_temp = nullptr;
    HIP_TRY(c, hipMalloc(&c->rows_temp, tb));
    c->rows_temp_bytes = tb;
  }
  RowsWork w = rows_views(c);
  int* dmap_d = c->rows_int + rows_int_need(c->rows_cap, c->rows_codes, c->rows_cids);
  HIP_TRY(c, hipMemcpyAsync(c->rows_ord, order, static_cast<size_t>(n) * sizeof(long long), hipMemcpyHostToDevice, st));
  if (keep) HIP_TRY(c, hipMemcpyAsync(c->rows_keep, keep, static_cast<size_t>(n), hipMemcpyHostToDevice, st));
  HIP_TRY(c, hipMemsetAsync(w.stat, 0, 4 * sizeof(int), st));
  HIP_TRY(c, hipMemsetAsync(w.err, 0, sizeof(int), st));
  // 1. the data list (prepare_data + mask_sequences2) and the read ranks (first appearance)
  long long mr[2] = {0, 0};
  HIP_TRY(c, rows_rank(w, n, c->rows_codes, c->rows_ord, keep ? c->rows_keep : nullptr, mr, st));
  const int64_t m = mr[0], n_reads = mr[1];
  {  // an order or qname code out of range ends the build here, before the grouping reads the ranks
    int err0 = 0;
    HIP_TRY(c, hipMemcpyAsync(&err0, w.err, sizeof(err0), hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipStreamSynchronize(st));
    if (err0 & kRowsErrOrder) return fail(c, FSLR_ERR_INVALID, "order holds a row out of range");
    if (err0 & kRowsErrCode) return fail(c, FSLR_ERR_INVALID, "qname code out of range");
  }
  if (m < 1) return fail(c, FSLR_ERR_INVALID, "no interval is left after the mask");
  if (n_reads >= FSLR_MAX_READS) return fail(c, FSLR_ERR_INVALID, "read count out of range");
  // 2. grouping into the CSR; the read lengths, gate values and the chromosomes present
  HIP_TRY(c, rows_csr(w, static_cast<int>(m), static_cast<int>(n_reads), c->rows_cids, st));
  int stat[4] = {0, 0, 0, 0}, err = 0;
  std::vector<int> present(static_cast<size_t>(c->rows_cids));
  HIP_TRY(c, hipMemcpyAsync(stat, w.stat, sizeof(stat), hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipMemcpyAsync(&err, w.err, sizeof(err), hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipMemcpyAsync(present.data(), w.present, present.size() * sizeof(int), hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipStreamSynchronize(st));
  info->n_reads = n_reads;
  info->n_intervals = m;
  info->max_len = stat[0];
  info->nal_varies = stat[1];
  if (err & kRowsErrOrder) return fail(c, FSLR_ERR_INVALID, "order holds a row out of range");
  if (err & kRowsErrCode) return fail(c, FSLR_ERR_INVALID, "qname code out of range");
  if (err & kRowsErrChrom) return fail(c, FSLR_ERR_INVALID, "chrom id out of range");
  if (err & kRowsErrCoord) return fail(c, FSLR_ERR_INVALID, "interval coordinates out of [0, 2^30)");
  if (err & kRowsErrNal) return fail(c, FSLR_ERR_INVALID, "n_alignments outside [0, 2^24)");
  if (err & kRowsErrQlen) return fail(c, FSLR_ERR_INVALID, "qlen2 outside [0, 2^31)");
  if (stat[0] > FSLR_MAX_L)
    return fail(c, FSLR_ERR_INVALID, "a read of more than FSLR_MAX_L intervals: set the reads with fslr_set_reads_any");
  // 3. dense chromosome ids (ascending numbers of the chromosomes present), thresholds, packing
  std::vector<int> dmap(static_cast<size_t>(c->rows_cids), 0);
  std::vector<int64_t> cid;
  for (int64_t k = 0; k < c->rows_cids; ++k)
    if (present[k]) {
      dmap[k] = static_cast<int>(cid.size());
      cid.push_back(k);
    }
  const int n_chroms = std::max<int>(1, static_cast<int>(cid.size()));
  info->n_chroms = n_chroms;
  if ((rc = ensure_capacity(c, n_reads, m, n_chroms))) return rc;
  if (n_chroms + 2 > c->upl64_cap) {
    if ((rc = dalloc(c, &c->upl64, static_cast<size_t>(n_chroms + 2)))) return rc;
    c->upl64_cap = n_chroms + 2;
  }
  HIP_TRY(c, hipMemcpyAsync(dmap_d, dmap.data(), dmap.size() * sizeof(int), hipMemcpyHostToDevice, st));
  // the dense ids go to w.val (the sort's input values, free after it) and the thresholds to thr_tmp
  int* ch_dense = w.val;
  HIP_TRY(c, rows_fold(w.aln_k, static_cast<int>(m), overlap, w.ch_raw, dmap_d, c->thr_tmp, ch_dense, w.stat, st));
  HIP_TRY(c, hipMemcpyAsync(c->data_pos, w.dp, static_cast<size_t>(m) * sizeof(int), hipMemcpyDeviceToDevice, st));
  unsigned long long* d_cnt = c->upl64;
  unsigned long long* d_err = c->upl64 + n_chroms;
  HIP_TRY(c, hipMemsetAsync(d_cnt, 0, static_cast<size_t>(n_chroms) * sizeof(unsigned long long), st));
  HIP_TRY(c, hipMemsetAsync(d_err, 0xff, 2 * sizeof(unsigned long long), st));
  UploadArgs ua{};
  ua.off = w.off;
  ua.qlen2 = w.q2;
  ua.nal = w.nal32;
  ua.chrom = ch_dense;
  ua.start = w.st32;
  ua.end = w.en32;
  ua.thr = c->thr_tmp;
  ua.dp = c->data_pos;
  ua.n = static_cast<int>(n_reads);
  ua.ni = static_cast<int>(m);
  ua.n_chroms = n_chroms;
  ua.reads_ok = true;
  ua.iv = c->iv;
  ua.rmeta = c->rmeta;
  ua.rlen8 = c->rlen8;
  ua.dch = c->dchrom;
  ua.drc = c->drec;
  ua.dgt = c->dgate;
  ua.inv = c->vals2;
  ua.chrom_cnt = d_cnt;
  ua.err = d_err;
  HIP_TRY(c, launch_upload_pack(ua, st));
  std::vector<int64_t> chrom_counts(static_cast<size_t>(n_chroms), 0);
  unsigned long long uerr[2] = {0, 0};
  HIP_TRY(c, hipMemcpyAsync(chrom_counts.data(), d_cnt, chrom_counts.size() * sizeof(int64_t), hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipMemcpyAsync(uerr, d_err, sizeof(uerr), hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipMemcpyAsync(stat, w.stat, sizeof(stat), hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipStreamSynchronize(st));
  c->reads_set = false;
  if (uerr[0] != ~0ull || uerr[1] != ~0ull) return fail(c, FSLR_ERR_STATE, "rows upload: inconsistent packing");
  info->general_thresholds = stat[2];
  info->any_zero_aln = stat[3];
  std::vector<unsigned char> zero(static_cast<size_t>(m), 0);
  if (stat[3]) {
    HIP_TRY(c, rows_zero_flags(c->thr_tmp, static_cast<int>(m), c->rows_keep, st));
    HIP_TRY(c, hipMemcpyAsync(zero.data(), c->rows_keep, zero.size(), hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipStreamSynchronize(st));
  }
  std::vector<int2> cr(static_cast<size_t>(n_chroms), make_int2(0, 0));
  int64_t acc = 0;
  for (int k = 0; k < n_chroms; ++k) {
    cr[k] = make_int2(static_cast<int>(acc), static_cast<int>(acc + chrom_counts[k]));
    acc += chrom_counts[k];
  }
  HIP_TRY(c, hipMemcpyAsync(c->crange, cr.data(), cr.size() * sizeof(int2), hipMemcpyHostToDevice, st));
  HIP_TRY(c, hipStreamSynchronize(st));
  c->have_data_pos = true;
  c->n = n_reads;
  c->ni = m;
  c->ni_idx = m;
  c->filter_active = false;
  c->chrom_counts.swap(chrom_counts);
  c->n_chroms = n_chroms;
  c->thr_mode = stat[2] ? 1 : 0;
  c->any_zero_aln = stat[3] != 0;
  c->aln_zero_host.swap(zero);
  c->rows_dmap.swap(dmap);
  c->rows_cid.swap(cid);
  c->rows_set = true;
  c->reads_set = true;
  ++c->reads_gen;
  c->pf_set = c->pf_on = false;
  c->index_built = false;
  c->lg_set = false;
  c->lg_perm.clear();
  c->edges_global = false;
  c->cap_gmode = false;
  ++c->input_gen;
  return FSLR_OK;
}

int fslr_get_read_codes(fslr_ctx* c, int64_t* codes) {
  if (!c || (!codes && c->n)) return FSLR_ERR_INVALID;
  if (!c->rows_set) return fail(c, FSLR_ERR_STATE, "the reads were not set by fslr_set_reads_rows");
  HIP_TRY(c, hipSetDevice(c->device));
  if (c->n)
    HIP_TRY(c, hipMemcpyAsync(codes, c->rows_l + c->rows_cap, static_cast<size_t>(c->n) * sizeof(int64_t),
                              hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FSLR_OK;
}

int fslr_get_csr(fslr_ctx* c, int32_t* read_off, int32_t* read_qlen2, int32_t* read_nal, int32_t* iv_chrom,
                 int32_t* iv_start, int32_t* iv_end, int64_t* iv_aln, int32_t* iv_thr, int64_t* data_pos,
                 int64_t* chrom_ids) {
  if (!c) return FSLR_ERR_INVALID;
  if (!c->rows_set) return fail(c, FSLR_ERR_STATE, "the reads were not set by fslr_set_reads_rows");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t st = c->stream;
  const RowsWork w = rows_views(c);
  const size_t nb = static_cast<size_t>(c->n) * sizeof(int), ib = static_cast<size_t>(c->ni) * sizeof(int);
  if (read_off) HIP_TRY(c, hipMemcpyAsync(read_off, w.off, nb + sizeof(int), hipMemcpyDeviceToHost, st));
  if (read_qlen2) HIP_TRY(c, hipMemcpyAsync(read_qlen2, w.q2, nb, hipMemcpyDeviceToHost, st));
  if (read_nal) HIP_TRY(c, hipMemcpyAsync(read_nal, w.nal32, nb, hipMemcpyDeviceToHost, st));
  if (iv_chrom) HIP_TRY(c, hipMemcpyAsync(iv_chrom, w.val, ib, hipMemcpyDeviceToHost, st));
  if (iv_start) HIP_TRY(c, hipMemcpyAsync(iv_start, w.st32, ib, hipMemcpyDeviceToHost, st));
  if (iv_end) HIP_TRY(c, hipMemcpyAsync(iv_end, w.en32, ib, hipMemcpyDeviceToHost, st));
  if (iv_thr) HIP_TRY(c, hipMemcpyAsync(iv_thr, c->thr_tmp, ib, hipMemcpyDeviceToHost, st));
  if (iv_aln) HIP_TRY(c, hipMemcpyAsync(iv_aln, w.aln_k, static_cast<size_t>(c->ni) * sizeof(int64_t),
                                        hipMemcpyDeviceToHost, st));
  std::vector<int> dp;
  if (data_pos) {
    dp.resize(static_cast<size_t>(c->ni));
    HIP_TRY(c, hipMemcpyAsync(dp.data(), w.dp, ib, hipMemcpyDeviceToHost, st));
  }
  HIP_TRY(c, hipStreamSynchronize(st));
  if (data_pos)
    for (int64_t k = 0; k < c->ni; ++k) data_pos[k] = dp[k];
  if (chrom_ids) std::copy(c->rows_cid.begin(), c->rows_cid.end(), chrom_ids);
  return FSLR_OK;
}

int fslr_fold_thresholds(fslr_ctx* c, double overlap) {
  if (!c) return FSLR_ERR_INVALID;
  if (!c->reads_set || !c->rows_set) return fail(c, FSLR_ERR_STATE, "the reads were not set by fslr_set_reads_rows");
  HIP_TRY(c, hipSetDevice(c->device));
  ++c->input_gen;
  const RowsWork w = rows_views(c);
  HIP_TRY(c, hipMemsetAsync(w.stat + 2, 0, 2 * sizeof(int), c->stream));
  HIP_TRY(c, rows_fold(w.aln_k, static_cast<int>(c->ni), overlap, nullptr, nullptr, c->thr_tmp, nullptr, w.stat,
                       c->stream));
  if (c->index_built && (c->built_n_shards != 1 || c->filter_active)) c->index_built = false;
  if (int rc = ensure_walk_index(c)) return rc;
  if (int rc = install_thresholds(c)) return rc;
  int stat[2] = {0, 0};
  HIP_TRY(c, hipMemcpyAsync(stat, w.stat + 2, sizeof(stat), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->thr_mode = stat[0] ? 1 : 0;
  return FSLR_OK;
}

}  // extern "C"

// the deferred edge-cap check: sticky host word 8 |= (max forward degree > thr) | (a listed
// ZeroDivisionError pair) << 1 — a repeat step that must not wait for the host (fslr_edge_cap_deferred)
__global__ void k_cap_sticky(const int* err, int thr, long long* sticky) {
  if (threadIdx.x == 0) {
    const long long f = (err[3] > thr ? 1 : 0) | (err[kErrZdCount] > 0 ? 2 : 0);
    if (f) *sticky |= f;
  }
}

extern "C" {

int fslr_edge_cap_deferred(fslr_ctx* c, int32_t thr) {
  if (!c) return FSLR_ERR_INVALID;
  if (!c->counters) return fail(c, FSLR_ERR_STATE, "no query has run");
  HIP_TRY(c, hipSetDevice(c->device));
  if (!c->sw_total) {
    HIP_TRY(c, hipHostMalloc(reinterpret_cast<void**>(&c->sw_total), 16 * sizeof(long long), hipHostMallocMapped));
    HIP_TRY(c, hipHostGetDevicePointer(reinterpret_cast<void**>(&c->sw_total_dev), c->sw_total, 0));
    c->sw_total[8] = 0;
  }
  k_cap_sticky<<<1, 64, 0, c->stream>>>(c->errw, thr, c->sw_total_dev + 8);
  HIP_TRY(c, hipGetLastError());
  return FSLR_OK;
}

int fslr_edge_cap_deferred_read(fslr_ctx* c, int32_t* flags) {
  if (!c || !flags) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  *flags = c->sw_total ? static_cast<int32_t>(c->sw_total[8]) : 0;
  if (c->sw_total) c->sw_total[8] = 0;
  return FSLR_OK;
}

int fslr_reserve_edges(fslr_ctx* c, int64_t capacity) {
  if (!c || capacity < 0) return FSLR_ERR_INVALID;
  c->hooked = false;
  HIP_TRY(c, hipSetDevice(c->device));
  if (capacity <= c->edge_cap) return FSLR_OK;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  int rc;
  if ((rc = dalloc(c, &c->edges, capacity)) || (rc = dalloc(c, &c->edge_iu, capacity))) return rc;
  c->edge_cap = capacity;
  return FSLR_OK;
}

int fslr_reserve_deferred(fslr_ctx* c, int64_t capacity) {
  if (!c || capacity < 0) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  if (capacity <= c->defer_cap) return FSLR_OK;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  int rc;
  if ((rc = dalloc(c, &c->defer, capacity))) return rc;
  c->defer_cap = capacity;
  return FSLR_OK;
}

int fslr_set_shard(fslr_ctx* c, int32_t shard, int32_t n_shards) {
  if (c) ++c->input_gen;
  if (!c) return FSLR_ERR_INVALID;
  if (n_shards < 1 || shard < 0 || shard >= n_shards) return fail(c, FSLR_ERR_INVALID, "bad shard");
  c->shard = shard;
  c->n_shards = n_shards;
  return FSLR_OK;
}

}  // extern "C"

static IndexBufs index_bufs(fslr_ctx* c) {
  IndexBufs b;
  b.rmeta = c->rmeta;
  b.iv = c->iv;
  b.shard = c->shard;
  b.n_shards = c->n_shards;
  b.dchrom = c->filter_active ? c->fdchrom : c->have_data_pos ? c->dchrom : nullptr;
  b.drec = c->filter_active ? c->fdrec : c->have_data_pos ? c->drec : nullptr;
  b.dgate = c->filter_active ? c->fdgate : c->dgate;
  b.data_pos = c->data_pos;
  b.chist = c->chist;
  b.keys = c->keys;
  b.keys2 = c->keys2;
  b.vals = c->vals;
  b.vals2 = c->vals2;
  b.s_start = c->s_start;
  b.endkey = c->endkey;
  b.pmaxkey = c->pmaxkey;
  b.temp = c->temp;
  b.temp_bytes = c->temp_bytes;
  b.crange = c->filter_active ? c->crange_f : c->crange;
  b.qpos = c->qpos;
  b.rng_s = c->rng_s;
  b.swin = c->swin;
  b.tile_tests = nullptr;
  b.idx4 = c->idx4;
  b.idx_gate = c->idx_gate;
  return b;
}

// edge count, error code and max forward degree of the last query, written by one tiny kernel into
// pinned host memory (no copy engine round trips); syncs
__global__ void k_peek(const unsigned long long* counters, const int* err, long long* out) {
  if (threadIdx.x == 0) {
    out[0] = static_cast<long long>(counters[kEdgeCount]);
    out[1] = err[0];
    out[2] = err[3];
    out[3] = err[kErrZdCount];
  }
}

int fslr::peek_counts(fslr_ctx* c, long long out[4]) {
  if (!c->sw_total) {
    HIP_TRY(c, hipHostMalloc(reinterpret_cast<void**>(&c->sw_total), 16 * sizeof(long long), hipHostMallocMapped));
    HIP_TRY(c, hipHostGetDevicePointer(reinterpret_cast<void**>(&c->sw_total_dev), c->sw_total, 0));
  }
  k_peek<<<1, 64, 0, c->stream>>>(c->counters, c->errw, c->sw_total_dev + 4);
  HIP_TRY(c, hipGetLastError());
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  const volatile long long* v = c->sw_total + 4;
  for (int k = 0; k < 4; ++k) out[k] = v[k];
  return FSLR_OK;
}

// a lean index (fslr_build_index for the sweep) gets its (chrom, end) keys (keys_only: what the
// backward ranges read, from its end column) or also its data -> sorted map (a full scatter again)
static int ensure_keys(fslr_ctx* c, bool keys_only) {
  if (!c->index_lean) return FSLR_OK;
  if (keys_only) {
    if (c->lean_keys) return FSLR_OK;
    HIP_TRY(c, launch_index_endkeys(index_bufs(c), static_cast<int>(c->ni_idx), c->built_n_chroms, c->stream));
    c->lean_keys = true;
    return FSLR_OK;
  }
  HIP_TRY(c, launch_index_rescatter(index_bufs(c), static_cast<int>(c->ni_idx), c->built_n_chroms, c->stream));
  c->index_lean = false;
  return FSLR_OK;
}

int fslr::ensure_bwd_ranges(fslr_ctx* c) {
  if (!c->index_built) return fail(c, FSLR_ERR_STATE, "fslr_build_index first");
  if (c->index_full || c->bwd_ranges) return FSLR_OK;
  if (int rc = ensure_keys(c, true)) return rc;
  HIP_TRY(c, launch_index_bwd_ranges(index_bufs(c), static_cast<int>(c->ni_idx), c->stream));
  c->bwd_ranges = true;
  return FSLR_OK;
}

int fslr::ensure_walk_index(fslr_ctx* c) {
  if (!c->index_built || c->index_full) return FSLR_OK;
  if (c->filter_active) return fail(c, FSLR_ERR_STATE, "the walk engine needs every chromosome's index");
  if (int rc = ensure_keys(c, false)) return rc;
  HIP_TRY(c, launch_index_walk_parts(index_bufs(c), static_cast<int>(c->n), static_cast<int>(c->ni), c->stream));
  c->index_full = true;
  return FSLR_OK;
}

extern "C" {

int fslr_build_index(fslr_ctx* c) {
  if (!c) return FSLR_ERR_INVALID;
  if (!c->reads_set) return fail(c, FSLR_ERR_STATE, "fslr_set_reads first");
  HIP_TRY(c, hipSetDevice(c->device));
  if (c->prof_phases) HIP_TRY(c, hipEventRecord(c->ev[0], c->stream));
  // the sweep engine's index only (the walk engine's parts follow on demand, ensure_walk_index)
  // where the data-order path applies and one context covers every query read
  const bool full = !c->filter_active && !(c->have_data_pos && c->n_chroms <= 64 && c->n_shards == 1);
  const int nch = c->filter_active ? c->n_chroms_f : c->n_chroms;
  IndexBufs ib = index_bufs(c);
  // the lean build also sums each 64-position tile's windows (the sweep plan's pair tests)
  const bool tt = !full && ib.dchrom && nch <= 64 && c->n_shards == 1;
  c->idx_tt_valid = false;
  if (tt) {
    const int64_t tiles = (c->ni_idx + 63) / 64 + 1;
    if (tiles > c->idx_tt_cap) {
      if (int rc = dalloc(c, &c->idx_tt, tiles)) return rc;
      c->idx_tt_cap = tiles;
    }
    ib.tile_tests = c->idx_tt;
  }
  HIP_TRY(c, launch_build_index(ib, static_cast<int>(c->n), static_cast<int>(c->ni_idx), nch, full, c->stream));
  c->idx_tt_valid = tt;
  c->index_lean = !full && index_bufs(c).dchrom && nch <= 64;
  c->lean_keys = false;
  c->built_n_chroms = nch;
  if (c->prof_phases) HIP_TRY(c, hipEventRecord(c->ev[1], c->stream));
  c->t_index_rec = c->prof_phases;
  c->index_built = true;
  c->index_full = full;
  c->bwd_ranges = full;
  c->built_shard = c->shard;
  c->built_n_shards = c->n_shards;
  return FSLR_OK;
}

static int query_impl(fslr_ctx* c, const fslr_params* p, int64_t a_begin, int64_t a_end, int shard, int n_shards);

int fslr_query(fslr_ctx* c, const fslr_params* p, int64_t a_begin, int64_t a_end) {
  if (!c || !p || !p->pass_table) return FSLR_ERR_INVALID;
  if (a_begin < 0 || a_end > c->n || a_begin > a_end) return fail(c, FSLR_ERR_INVALID, "bad read range");
  if (c->index_built && c->built_n_shards != 1)
    return fail(c, FSLR_ERR_STATE, "index built for one shard (fslr_set_shard): use fslr_query_shard");
  return query_impl(c, p, a_begin, a_end, 0, 1);
}

int fslr_query_shard(fslr_ctx* c, const fslr_params* p, int32_t shard, int32_t n_shards) {
  if (!c || !p || !p->pass_table) return FSLR_ERR_INVALID;
  if (n_shards < 1 || shard < 0 || shard >= n_shards) return fail(c, FSLR_ERR_INVALID, "bad shard");
  if (c->index_built && c->built_n_shards != 1 && (c->built_shard != shard || c->built_n_shards != n_shards))
    return fail(c, FSLR_ERR_STATE, "index built for another shard");
  return query_impl(c, p, 0, c->n, shard, n_shards);
}

// The position-sweep engine (sweep.hip).  One pass: the sweep writes each tile's entries at an
// upper-bound slot (its pair tests, scanned); one sync reads the entry count, the upper-bound total
// and an overflow flag from pinned host memory the kernels write; the tiles are packed, grouped by
// A and evaluated.  A too-small upper-bound buffer is grown and the sweep rerun (first query on an
// input); an upper bound beyond the budget (half the free HBM, at least 8 GB) takes the two-pass
// fallback (count, then emit: the sweep runs twice).
static int sweep_front(fslr_ctx* c, const fslr_params* p, int64_t a_begin, int64_t a_end, hipEvent_t e0,
                       hipEvent_t e1, SweepArgs& s, int& mode, bool defer = false, bool coarse = false,
                       bool count_only = false, int dest_n = 0, int dest_shift = 0) {
  // upper-bound slots (8 B each) the one-pass sweep may use: half the free HBM, at least 2^30; asked
  // only when the slot buffer has to grow (hipMemGetInfo is a driver round trip, kept off repeat queries)
  auto ub_budget = []() {
    int64_t b = int64_t(1) << 30;
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess)
      b = std::max<int64_t>(b, static_cast<int64_t>(fr / 2 / sizeof(unsigned long long)));
    return b;
  };
  const int64_t nix = c->ni_idx;                      // positions of the (possibly chromosome-filtered) index
  const int64_t tiles = (nix + 63) / 64 + 1;
  int rc;
  if (tiles > c->sw_tiles) {
    if ((rc = dalloc(c, &c->sw_tile, 4 * tiles))) return rc;
    c->sw_tiles = tiles;
    c->ent_cap = 0;                                  // re-size the scan scratch with the entries
  }
  if (!c->sw_total) {
    HIP_TRY(c, hipHostMalloc(reinterpret_cast<void**>(&c->sw_total), 16 * sizeof(long long), hipHostMallocMapped));
    HIP_TRY(c, hipHostGetDevicePointer(reinterpret_cast<void**>(&c->sw_total_dev), c->sw_total, 0));
  }
  if (!c->sw_wstat) {
    const int w = sweep_max_waves();
    if ((rc = dalloc(c, &c->sw_wstat, static_cast<size_t>(w) * 4))) return rc;
    if ((rc = dalloc(c, &c->sw_wlo, static_cast<size_t>(w) + 1))) return rc;
    c->sw_wstat_waves = w;
  }
  if (c->ent_cap == 0 && (rc = reserve_entries(c, std::max<int64_t>(1 << 20, nix)))) return rc;
  if (c->ent_ub_cap == 0) {
    if ((rc = dalloc(c, &c->ent_ub, std::max<int64_t>(1 << 20, 4 * nix)))) return rc;
    c->ent_ub_cap = std::max<int64_t>(1 << 20, 4 * nix);
  }
  if ((rc = ensure_grp(c))) return rc;
  s.grp = c->grp;
  s.rmeta = c->rmeta;
  s.rlen8 = c->rlen8;
  s.idx4 = c->idx4;
  s.idx_gate = c->idx_gate;
  s.rng_s = c->rng_s;
  s.swin = c->swin;
  s.umax = c->umax;
  s.ni = static_cast<int>(nix);
  if (c->filter_active && c->pf_on && c->pf_thr_gen != c->thr_gen)     // the halo ends at the old windows
    return fail(c, FSLR_ERR_STATE, "the thresholds changed after fslr_set_position_filter: plan the range again");
  s.nq = c->filter_active && c->pf_on ? static_cast<int>(c->pf_hi - c->pf_lo) : static_cast<int>(nix);
  s.n_reads = static_cast<int>(c->n);
  s.a_begin = static_cast<int>(a_begin);
  s.a_end = static_cast<int>(a_end);
  s.qlen_cut = p->qlen_cut;
  s.nal_cut = p->nal_cut;
  s.lb = c->lbounds;
  s.tile_cnt = c->sw_tile;
  s.tile_off = c->sw_tile + c->sw_tiles;
  // the lean index build summed the tiles' windows already, unless a position filter's query range ends
  // inside the index (its last query tile then holds fewer positions than the index tile)
  s.tests_ready = c->idx_tt_valid && s.nq == static_cast<int>(nix);
  s.tile_tests = s.tests_ready ? c->idx_tt : c->sw_tile + 2 * c->sw_tiles;
  s.tile_ub = c->sw_tile + 3 * c->sw_tiles;
  s.edges = c->edges;
  s.edge_iu = c->edge_iu;
  s.edge_cap = c->edge_cap;
  s.fwd = c->fwd;
  s.counters = c->counters;
  s.err = c->errw;
  s.wstat = c->sw_wstat;
  s.wstat_waves = c->sw_wstat_waves;
  s.wlo = c->sw_wlo;
  s.n_ent = 0;
  s.n_dev = nullptr;
  s.ent_cap = c->ent_cap;
  for (int k = 0; k < 5; ++k) s.ev[k] = c->prof_phases ? c->sw_ev[k] : nullptr;
  s.ev[0] = nullptr;                                // recorded here, around the sweep pass
  s.hist_mat = nullptr;
  s.hist_mod = 0;
  if (coarse) sweep_coarse_hist(s);                  // the sweep counts the grouping's coarse buckets
  if (dest_n > 0) sweep_dest_hist(s, dest_n, dest_shift);   // ... or a partition's destinations
  s.dest_totals = dest_n > 0 ? c->part_cnt : nullptr;
  // the gate ranges depend on the reads and the two cuts only: a repeat query keeps them
  if (!c->reuse || c->lb_gen != c->input_gen || c->lb_q != p->qlen_cut || c->lb_n != p->nal_cut) {
    HIP_TRY(c, launch_len_bounds(c->rmeta, 0, static_cast<int>(c->n), p->qlen_cut, p->nal_cut, c->lbounds, c->stream));
    c->lb_gen = c->input_gen;
    c->lb_q = p->qlen_cut;
    c->lb_n = p->nal_cut;
  }
  mode = count_only ? 0 : 2;                         // count_only: per-tile entry counts, no slots
  for (int attempt = 0; attempt < 3; ++attempt) {
    s.ent = c->ent;
    s.ent_sorted = c->ent_sorted;
    s.ent_ub = c->ent_ub;
    s.ub_cap = c->ent_ub_cap;
    s.temp = c->sweep_temp;
    s.temp_bytes = c->sweep_temp_bytes;
    if (mode == 2) HIP_TRY(c, launch_sweep_plan(s, c->stream));
    s.k0 = e0;                                       // the pair-kernel ring: the sweep kernel alone
    s.k1 = e1;
    s.p0 = s.p1 = nullptr;
    if (c->prof_phases) HIP_TRY(c, hipEventRecord(c->sw_ev[0], c->stream));
    // a repeat of the last synchronous query on unchanged input: same entry count, no readback
    const bool fast = c->reuse && !defer && mode == 2 && attempt == 0 && c->sw_prev_gen == c->input_gen &&
                      c->sw_prev_a0 == a_begin && c->sw_prev_a1 == a_end && c->sw_prev_q == p->qlen_cut &&
                      c->sw_prev_nc == p->nal_cut && c->sw_prev_umax == c->umax_host && c->sw_prev_n > 0 &&
                      c->sw_prev_n <= c->ent_cap && c->sw_prev_n < (int64_t(1) << 31) && !c->filter_active;
    long long* n_dev = reinterpret_cast<long long*>(c->counters + kSwNdev);
    HIP_TRY(c, launch_sweep_count(s, mode, c->sw_total_dev, c->stream, fast ? n_dev : nullptr,
                                  fast ? c->ent_cap : -1));
    c->sw_fast_used = fast;
    if (fast) {
      s.n_ent = c->sw_prev_n;                        // grid shapes; the kernels read the count at n_dev
      s.n_dev = n_dev;
      break;
    }
    if (defer) {                                     // the caller reads the counts and flags later
      s.n_ent = -1;
      return FSLR_OK;
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    const volatile long long* tot = c->sw_total;
    if (mode == 2 && (tot[2] & 8)) {
      // upper-bound buffer too small (or beyond the budget: two passes); clear the flag and counters
      const int64_t need = tot[1];
      if (need > ub_budget()) {
        mode = 0;
      } else {
        if ((rc = dalloc(c, &c->ent_ub, need + (need >> 3) + 4096))) return rc;
        c->ent_ub_cap = need + (need >> 3) + 4096;
      }
      HIP_TRY(c, hipMemsetAsync(c->counters, 0, kNumCounters * sizeof(unsigned long long), c->stream));
      HIP_TRY(c, hipMemsetAsync(c->errw, 0, kErrSticky * sizeof(int), c->stream));
      continue;
    }
    s.n_ent = tot[0];
    if (mode == 2 && !c->filter_active) {            // remember the input: the next identical query skips the sync
      c->sw_prev_gen = c->input_gen;
      c->sw_prev_a0 = a_begin;
      c->sw_prev_a1 = a_end;
      c->sw_prev_q = p->qlen_cut;
      c->sw_prev_nc = p->nal_cut;
      c->sw_prev_umax = c->umax_host;
      c->sw_prev_n = s.n_ent;
    }
    break;
  }
  if (s.n_ent > c->ent_cap && (rc = reserve_entries(c, s.n_ent + (s.n_ent >> 3) + 4096))) return rc;
  s.ent = c->ent;
  s.ent_sorted = c->ent_sorted;
  s.ent_cap = c->ent_cap;
  s.temp = c->sweep_temp;
  s.temp_bytes = c->sweep_temp_bytes;
  return FSLR_OK;
}

static int sweep_impl(fslr_ctx* c, const fslr_params* p, int64_t a_begin, int64_t a_end, hipEvent_t e0,
                      hipEvent_t e1) {
  SweepArgs s{};
  int mode = 2;
  int rc = sweep_front(c, p, a_begin, a_end, e0, e1, s, mode, false, true);
  if (rc) return rc;
  if (e0) {                                          // profiling: the pair-stage kernel's ring too
    const int slot = static_cast<int>(c->n_kern2++ % fslr_ctx::kKernRing);
    s.p0 = c->kev2[2 * slot];
    s.p1 = c->kev2[2 * slot + 1];
  }
  s.parent = c->parent;                              // the edges hook the union-find as they are formed
  HIP_TRY(c, launch_sweep_pairs(s, mode, c->stream));
  c->hooked = true;
  c->sw_ev_rec = c->prof_phases;
  return FSLR_OK;
}

// buffers, the folded cut table and cleared counters / errors / forward degrees for one query
// keep_sticky: the repeat-partition flags (kErrSticky) and the ZeroDivisionError pairs of the partition
// (kErrZdCount) survive (a repeat partition and the
// evaluations after it); any other query starts a new series and clears them
static int prepare_query(fslr_ctx* c, const fslr_params* p, bool keep_sticky = false) {
  HIP_TRY(c, hipSetDevice(c->device));
  if (c->edge_cap == 0) {
    int rc = fslr_reserve_edges(c, std::max<int64_t>(1 << 16, 12 * c->n));
    if (rc) return rc;
  }
  if (c->defer_cap == 0) {
    int rc = fslr_reserve_deferred(c, std::max<int64_t>(1 << 20, c->n));
    if (rc) return rc;
  }
  // I/U >= cut(I) is monotone in U (fl(I/U) never increases with U): fold each row of the pass
  // table into its largest passing U; reject tables that are not of that form
  c->umax_host.assign(FSLR_MAX_L, 0);
  for (int I = 1; I <= FSLR_MAX_L; ++I) {
    const unsigned char* row = p->pass_table + (I - 1) * kPassStride;
    int um = 0;
    for (int U = I; U <= kPassStride; ++U)
      if (row[U - 1]) um = U;
    for (int U = I; U <= um; ++U)
      if (!row[U - 1]) return fail(c, FSLR_ERR_INVALID, "pass_table row is not a prefix in U");
    c->umax_host[I - 1] = um;
  }
  if (c->umax_host != c->umax_dev_copy) {
    c->umax_dev_copy = c->umax_host;
    HIP_TRY(c, hipMemcpyAsync(c->umax, c->umax_dev_copy.data(), FSLR_MAX_L * sizeof(int), hipMemcpyHostToDevice,
                              c->stream));
  }
  if (!c->wstat) {
    const int w = query_max_waves();
    int rc = dalloc(c, &c->wstat, static_cast<size_t>(w) * kWStride);
    if (rc) return rc;
    c->wstat_waves = w;
  }
  HIP_TRY(c, launch_query_reset(c->counters, kNumCounters, c->errw, keep_sticky ? kErrKeep : kErrWords, c->fwd,
                                c->parent, static_cast<int>(c->n), c->stream));
  c->hooked = false;
  std::memset(&c->cap_stats, 0, sizeof(c->cap_stats));
  if (!keep_sticky) c->zd_lost = false;             // a new series lists its pairs from the start
  c->edges_global = false;
  c->cap_gmode = false;
  c->last_qcut = p->qlen_cut;                       // the cap replay's pair predicate
  c->last_ncut = p->nal_cut;
  c->q_thr = p->edge_threshold;
  c->zd_host = true;                                // fslr_query clears it: there the library decides
  return FSLR_OK;
}

static int query_impl(fslr_ctx* c, const fslr_params* p, int64_t a_begin, int64_t a_end, int shard, int n_shards) {
  if (!c->index_built) return fail(c, FSLR_ERR_STATE, "fslr_build_index first");
  if (c->filter_active)
    return fail(c, FSLR_ERR_STATE, "the index covers a chromosome subset (fslr_set_chrom_filter): use "
                                   "fslr_sweep_partition / fslr_sweep_evaluate");
  if (int rc = prepare_query(c, p)) return rc;
  c->zd_host = n_shards > 1;                        // a query shard: the caller decides over every shard
  QueryArgs g;
  g.rmeta = c->rmeta;
  g.iv = c->iv;
  g.qpos = c->qpos;
  g.rng_s = c->rng_s;
  g.idx4 = c->idx4;
  g.idx_gate = c->idx_gate;
  g.defer = c->defer;
  g.defer_cap = c->defer_cap;
  g.umax = c->umax;
  g.lb = c->lbounds;
  c->lb_gen = -1;                                    // the walk engine writes its own range of lbounds
  g.qlen_cut = p->qlen_cut;
  g.nal_cut = p->nal_cut;
  g.a_begin = static_cast<int>(a_begin);
  g.a_end = static_cast<int>(a_end);
  g.shard = shard;
  g.n_shards = n_shards;
  g.edges = c->edges;
  g.edge_iu = c->edge_iu;
  g.edge_cap = c->edge_cap;
  g.fwd = c->fwd;
  g.heavy = c->heavy;
  g.counters = c->counters;
  g.err = c->errw;
  g.mode = c->ablate & 3;                            // bits 0-1: the walk kernel's ablations
  g.diag = c->diag;
  g.wstat = c->wstat;
  g.wstat_waves = c->wstat_waves;
  g.ev_k0 = g.ev_k1 = nullptr;
  if (c->profiling && c->n > 0 && a_end > a_begin) {
    const int slot = static_cast<int>(c->n_kern++ % fslr_ctx::kKernRing);
    g.ev_k0 = c->kev[2 * slot];
    g.ev_k1 = c->kev[2 * slot + 1];
  }
  c->last_full = a_begin == 0 && a_end == c->n && n_shards == 1;
  c->last_qcut = p->qlen_cut;
  c->last_ncut = p->nal_cut;
  const int want = p->flags & 3;
  const bool sweep_ok = c->thr_mode == 0 && !c->any_zero_aln && n_shards == 1;
  if (want == FSLR_ENGINE_SWEEP && !sweep_ok)
    return fail(c, FSLR_ERR_INVALID, "the sweep engine needs overlap thresholds >= 1, no aln_size == 0 interval "
                                     "and one query shard");
  const bool sweep = want == FSLR_ENGINE_SWEEP || (want == FSLR_ENGINE_AUTO && sweep_ok && c->last_full);
  c->last_engine = sweep ? FSLR_ENGINE_SWEEP : FSLR_ENGINE_WALK;
  if (c->prof_phases) HIP_TRY(c, hipEventRecord(c->ev[2], c->stream));
  if (!sweep) {
    int rc = ensure_walk_index(c);
    if (rc) return rc;
  }
  if (sweep) {
    int rc = sweep_impl(c, p, a_begin, a_end, g.ev_k0, g.ev_k1);
    if (rc) return rc;
  } else {
    HIP_TRY(c, launch_query(g, c->thr_mode, c->stream));
  }
  if (c->prof_phases) HIP_TRY(c, hipEventRecord(c->ev[3], c->stream));
  c->t_query_rec = c->prof_phases;
  c->t_kernel_rec = c->profiling && c->n > 0 && a_end > a_begin;
  return FSLR_OK;
}

// ---- multi-GPU sweep: chromosome-filtered index, entry partition by owner, owner evaluation ----
int fslr_set_chrom_filter(fslr_ctx* c, const uint8_t* owned) {
  if (c) c->pf_on = false;
  if (c) ++c->input_gen;
  if (!c) return FSLR_ERR_INVALID;
  if (!c->reads_set) return fail(c, FSLR_ERR_STATE, "fslr_set_reads first");
  HIP_TRY(c, hipSetDevice(c->device));
  c->index_built = false;
  if (!owned) {
    c->filter_active = false;
    c->ni_idx = c->ni;
    return FSLR_OK;
  }
  if (!c->have_data_pos)
    return fail(c, FSLR_ERR_INVALID, "a chromosome filter needs the start-sorted data order (iv_data_pos)");
  // the owned chromosomes are renumbered 0 .. k-1 (chromosome order) in the filtered index: the
  // counting-sort build applies whenever a rank owns at most 64 of them, however many there are
  std::vector<int2> cr;
  std::vector<int> lmap(static_cast<size_t>(c->n_chroms), -1);
  int64_t acc = 0;
  for (int ch = 0; ch < c->n_chroms; ++ch) {
    if (!owned[ch]) continue;
    lmap[ch] = static_cast<int>(cr.size());
    const int64_t k = c->chrom_counts[ch];
    cr.push_back(make_int2(static_cast<int>(acc), static_cast<int>(acc + k)));
    acc += k;
  }
  const int64_t nf = acc;
  int rc;
  if (nf > c->f_cap) {
    if ((rc = dalloc(c, &c->fdchrom, nf)) || (rc = dalloc(c, &c->fdrec, nf)) || (rc = dalloc(c, &c->fdgate, nf)))
      return rc;
    c->f_cap = nf;
  }
  if (static_cast<int64_t>(std::max<size_t>(cr.size(), 1)) > c->crange_f_cap) {
    if ((rc = dalloc(c, &c->crange_f, std::max<size_t>(cr.size(), 1)))) return rc;
    c->crange_f_cap = static_cast<int64_t>(std::max<size_t>(cr.size(), 1));
  }
  if (c->n_chroms > c->fmap_cap) {
    if ((rc = dalloc(c, &c->fmap, static_cast<size_t>(c->n_chroms)))) return rc;
    c->fmap_cap = c->n_chroms;
  }
  if (!cr.empty())
    HIP_TRY(c, hipMemcpyAsync(c->crange_f, cr.data(), cr.size() * sizeof(int2), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipMemcpyAsync(c->fmap, lmap.data(), lmap.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, launch_chrom_filter(c->dchrom, c->drec, c->dgate, c->fmap, static_cast<int>(c->ni), c->fdchrom, c->fdrec,
                                 c->fdgate, c->vals2, c->vals, c->temp, c->temp_bytes, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->filter_active = true;
  c->n_chroms_f = static_cast<int>(cr.size());
  c->ni_idx = nf;
  return FSLR_OK;
}

// ---- the position split (multi-GPU) ----------------------------------------------------
int fslr_position_costs(fslr_ctx* c, int64_t* tests, int64_t* reach, int64_t n_tiles) {
  if (!c || !tests || !reach) return FSLR_ERR_INVALID;
  if (!c->index_built || c->filter_active) return fail(c, FSLR_ERR_STATE, "fslr_build_index over every chromosome first");
  const int64_t nt = (c->ni + 63) / 64;
  if (n_tiles != nt) return fail(c, FSLR_ERR_INVALID, "n_tiles must be ceil(n_intervals / 64)");
  HIP_TRY(c, hipSetDevice(c->device));
  if (2 * std::max<int64_t>(nt, 1) > c->pf_cost_cap) {
    if (int rc = dalloc(c, &c->pf_cost, 2 * std::max<int64_t>(nt, 1))) return rc;
    c->pf_cost_cap = 2 * std::max<int64_t>(nt, 1);
  }
  HIP_TRY(c, launch_tile_costs(c->swin, static_cast<int>(c->ni), c->pf_cost, c->pf_cost + nt, c->stream));
  if (nt) {
    HIP_TRY(c, hipMemcpyAsync(tests, c->pf_cost, nt * sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipMemcpyAsync(reach, c->pf_cost + nt, nt * sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FSLR_OK;
}

int fslr_position_entries(fslr_ctx* c, const fslr_params* p, int64_t* entries, int64_t n_tiles) {
  if (!c || !p || !p->pass_table || !entries) return FSLR_ERR_INVALID;
  if (!c->index_built || c->filter_active) return fail(c, FSLR_ERR_STATE, "fslr_build_index over every chromosome first");
  const int64_t nt = (c->ni + 63) / 64;
  if (n_tiles != nt) return fail(c, FSLR_ERR_INVALID, "n_tiles must be ceil(n_intervals / 64)");
  if (c->thr_mode != 0 || c->any_zero_aln)
    return fail(c, FSLR_ERR_INVALID, "the sweep engine needs overlap thresholds >= 1 and no aln_size == 0 interval");
  if (int rc = prepare_query(c, p)) return rc;
  SweepArgs s{};
  int mode = 0;
  if (int rc = sweep_front(c, p, 0, c->n, nullptr, nullptr, s, mode, false, false, true)) return rc;
  if (nt) HIP_TRY(c, hipMemcpyAsync(entries, s.tile_cnt, nt * sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->last_full = false;                               // no graph from this sweep
  return FSLR_OK;
}

namespace {
// activate the kept selection: its records in data order, renumbered, as the filtered index's input
int pos_activate(fslr_ctx* c) {
  const int64_t m = c->pf_end - c->pf_lo;
  const int nch = static_cast<int>(c->pf_cr.size());
  if (std::max<int64_t>(nch, 1) > c->crange_f_cap) {
    if (int rc = dalloc(c, &c->crange_f, std::max<int64_t>(nch, 1))) return rc;
    c->crange_f_cap = std::max<int64_t>(nch, 1);
  }
  if (m > c->f_cap) {
    int rc;
    if ((rc = dalloc(c, &c->fdchrom, m)) || (rc = dalloc(c, &c->fdrec, m)) || (rc = dalloc(c, &c->fdgate, m))) return rc;
    c->f_cap = m;
  }
  if (nch) HIP_TRY(c, hipMemcpyAsync(c->crange_f, c->pf_cr.data(), nch * sizeof(int2), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, launch_pos_gather(c->pf_sel, static_cast<int>(m), c->dchrom, c->drec, c->dgate, c->pf_lmap, c->fdchrom,
                               c->fdrec, c->fdgate, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->filter_active = true;
  c->pf_on = true;
  c->n_chroms_f = nch;
  c->ni_idx = m;
  c->index_built = false;
  ++c->input_gen;
  return FSLR_OK;
}
}  // namespace

int fslr_set_position_filter(fslr_ctx* c, int64_t lo, int64_t hi, int64_t end) {
  if (!c || lo < 0 || hi < lo || end < hi) return FSLR_ERR_INVALID;
  if (!c->reads_set) return fail(c, FSLR_ERR_STATE, "fslr_set_reads first");
  if (end > c->ni) return fail(c, FSLR_ERR_INVALID, "position range beyond the index");
  if (!c->have_data_pos || c->n_chroms > 64 || c->n_shards != 1)
    return fail(c, FSLR_ERR_STATE, "the position split needs the data-order index build (iv_data_pos, <= 64 chromosomes)");
  HIP_TRY(c, hipSetDevice(c->device));
  // the full index once more, with its data -> sorted map (vals)
  c->filter_active = c->pf_on = false;
  c->ni_idx = c->ni;
  if (int rc = fslr_build_index(c)) return rc;
  if (int rc = ensure_keys(c, false)) return rc;
  const int64_t m = end - lo;
  if (std::max<int64_t>(m, 1) > c->pf_sel_cap) {
    if (int rc = dalloc(c, &c->pf_sel, std::max<int64_t>(m, 1))) return rc;
    c->pf_sel_cap = std::max<int64_t>(m, 1);
  }
  if (c->n_chroms > c->pf_lmap_cap) {
    if (int rc = dalloc(c, &c->pf_lmap, c->n_chroms)) return rc;
    c->pf_lmap_cap = c->n_chroms;
  }
  // the chromosomes the range meets, numbered in order, and their ranges inside it
  std::vector<int> lmap(static_cast<size_t>(c->n_chroms), -1);
  std::vector<int2> cr;
  int64_t acc = 0;
  for (int ch = 0; ch < c->n_chroms; ++ch) {
    const int64_t a = acc, b = acc + c->chrom_counts[ch];
    acc = b;
    const int64_t x = std::max(a, lo), y = std::min(b, end);
    if (x >= y) continue;
    lmap[ch] = static_cast<int>(cr.size());
    cr.push_back(make_int2(static_cast<int>(x - lo), static_cast<int>(y - lo)));
  }
  HIP_TRY(c, hipMemcpyAsync(c->pf_lmap, lmap.data(), lmap.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, launch_pos_select(c->vals, static_cast<int>(c->ni), static_cast<int>(lo), static_cast<int>(end), c->vals2,
                               c->qpos, c->pf_sel, c->temp, c->temp_bytes, c->stream));
  c->index_full = false;                                          // qpos was scratch: the walk parts are gone
  c->pf_lo = lo;
  c->pf_hi = hi;
  c->pf_end = end;
  c->pf_cr.swap(cr);
  c->pf_set = true;
  c->pf_gen = c->reads_gen;
  c->pf_thr_gen = c->thr_gen;
  return pos_activate(c);
}

int fslr_use_position_filter(fslr_ctx* c) {
  if (!c) return FSLR_ERR_INVALID;
  if (!c->pf_set || c->pf_gen != c->reads_gen) return fail(c, FSLR_ERR_STATE, "no position filter for these reads");
  HIP_TRY(c, hipSetDevice(c->device));
  return pos_activate(c);
}

int fslr_sweep_partition(fslr_ctx* c, const fslr_params* p, int32_t n_dest, int32_t block_shift, void* dst,
                         int64_t dst_cap, int64_t* counts) {
  if (!c || !p || !p->pass_table || n_dest < 1 || n_dest > kMaxDest || block_shift < 0 || block_shift > 24 ||
      !counts || dst_cap < 0 || (!dst && dst_cap))
    return FSLR_ERR_INVALID;
  if (!c->index_built) return fail(c, FSLR_ERR_STATE, "fslr_build_index first");
  if (c->thr_mode != 0 || c->any_zero_aln)
    return fail(c, FSLR_ERR_INVALID, "the sweep engine needs overlap thresholds >= 1 and no aln_size == 0 interval");
  if (int rc = prepare_query(c, p)) return rc;
  c->last_full = false;
  c->last_engine = FSLR_ENGINE_SWEEP;
  if (!c->part_cnt && dalloc(c, &c->part_cnt, kMaxDest)) return FSLR_ERR_NOMEM;
  long long* totals = c->part_cnt;
  auto* out = static_cast<unsigned long long*>(dst);
  long long tot[kMaxDest];
  int ew[kErrWords] = {};
  auto read_back = [&]() -> int {
    HIP_TRY(c, hipMemcpyAsync(tot, totals, n_dest * sizeof(long long), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipMemcpyAsync(ew, c->errw, sizeof(ew), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return FSLR_OK;
  };
  // one sync: the sweep writes its tile slots, the partition reads them straight into dst; the
  // slot-overflow flag is checked at the end (first call on an input: grow, rerun synchronously)
  hipEvent_t k0 = nullptr, k1 = nullptr;           // the pair-kernel ring: the sweep kernel
  if (c->profiling && c->n > 0) {
    const int slot = static_cast<int>(c->n_kern++ % fslr_ctx::kKernRing);
    k0 = c->kev[2 * slot];
    k1 = c->kev[2 * slot + 1];
  }
  SweepArgs s{};
  int mode = 2;
  if (int rc = sweep_front(c, p, 0, c->n, k0, k1, s, mode, true, false, false, n_dest, block_shift)) return rc;
  HIP_TRY(c, launch_sweep_partition(s, 2, block_shift, n_dest, out, dst_cap, totals, c->stream));
  if (int rc = read_back()) return rc;
  const volatile long long* st = c->sw_total;
  if (st[2] & 8) {
    if (int rc = prepare_query(c, p)) return rc;
    mode = 2;
    if (int rc = sweep_front(c, p, 0, c->n, k0, k1, s, mode, false, false, false, n_dest, block_shift)) return rc;
    if (mode == 0) HIP_TRY(c, launch_sweep_dense(s, 0, c->stream));     // dense entries in `ent`
    HIP_TRY(c, launch_sweep_partition(s, mode, block_shift, n_dest, out, dst_cap, totals, c->stream));
    if (int rc = read_back()) return rc;
  }
  c->t_kernel_rec = k0 != nullptr;
  // ZeroDivisionError pairs are listed (ew[kErrZdCount]), not raised: the caller decides once the edge
  // cap's binding is known over every rank (fslr_read_stats zd_pairs)
  int64_t sum = 0;
  for (int k = 0; k < n_dest; ++k) sum += (counts[k] = tot[k]);
  c->pt_gen = 0;
  if (sum > dst_cap) return fail(c, FSLR_ERR_STATE, "destination buffer too small for the entries (see counts)");
  // clean, and one pass into the upper-bound slots (a two-pass rerun left them undersized): a repeat
  // may replay this partition
  if (ew[kErrOverflow] == 0 && mode == 2) {
    c->pt_gen = c->input_gen;
    c->pt_q = p->qlen_cut;
    c->pt_nc = p->nal_cut;
    c->pt_umax = c->umax_host;
    c->pt_ndest = n_dest;
    c->pt_shift = block_shift;
    c->pt_sum = sum;
    c->pt_counts.assign(tot, tot + n_dest);
  }
  return FSLR_OK;
}

// a repeat partition's destination totals against the last synchronous one's: a difference flags
// the query (overflow_flags 32), whose results are then refused by fslr_read_stats
struct PartExpect {
  long long n[kMaxDest];
};
__global__ void k_part_check(const long long* __restrict__ totals, PartExpect expect, int n_dest, int* err) {
  const int k = threadIdx.x;
  if (k < n_dest && totals[k] != expect.n[k]) atomicOr(&err[kErrSticky], 32);
}

int fslr_sweep_partition_repeat(fslr_ctx* c, const fslr_params* p, int32_t n_dest, int32_t block_shift, void* dst,
                                int64_t dst_cap) {
  if (!c || !p || !p->pass_table || n_dest < 1 || n_dest > kMaxDest || !dst) return FSLR_ERR_INVALID;
  if (!c->index_built) return fail(c, FSLR_ERR_STATE, "fslr_build_index first");
  if (int rc = prepare_query(c, p, true)) return rc;     // folds the cut table into umax_host
  if (c->pt_gen != c->input_gen || c->pt_q != p->qlen_cut || c->pt_nc != p->nal_cut || c->pt_umax != c->umax_host ||
      c->pt_ndest != n_dest || c->pt_shift != block_shift || c->pt_sum > dst_cap)
    return fail(c, FSLR_ERR_STATE, "no synchronous fslr_sweep_partition of this input, parameters and split");
  c->last_full = false;
  c->last_engine = FSLR_ENGINE_SWEEP;
  hipEvent_t k0 = nullptr, k1 = nullptr;
  if (c->profiling && c->n > 0) {
    const int slot = static_cast<int>(c->n_kern++ % fslr_ctx::kKernRing);
    k0 = c->kev[2 * slot];
    k1 = c->kev[2 * slot + 1];
  }
  SweepArgs s{};
  int mode = 2;
  if (int rc = sweep_front(c, p, 0, c->n, k0, k1, s, mode, true, false, false, n_dest, block_shift)) return rc;
  HIP_TRY(c, launch_sweep_partition(s, 2, block_shift, n_dest, static_cast<unsigned long long*>(dst), dst_cap,
                                    c->part_cnt, c->stream));
  PartExpect ex{};
  for (int k = 0; k < n_dest; ++k) ex.n[k] = c->pt_counts[k];
  if (c->ablate & 64) ex.n[0] += 1;                     // tests: a repeat whose totals differ
  k_part_check<<<1, kMaxDest, 0, c->stream>>>(c->part_cnt, ex, n_dest, c->errw);
  HIP_TRY(c, hipGetLastError());
  c->t_kernel_rec = k0 != nullptr;
  return FSLR_OK;
}

int fslr_sweep_evaluate(fslr_ctx* c, const fslr_params* p, const void* entries, int64_t n) {
  if (!c || !p || !p->pass_table || (!entries && n) || n < 0) return FSLR_ERR_INVALID;
  if (!c->reads_set) return fail(c, FSLR_ERR_STATE, "fslr_set_reads first");
  if (int rc = prepare_query(c, p, true)) return rc;
  if (n > c->ent_cap && reserve_entries(c, n + (n >> 3) + 4096)) return FSLR_ERR_NOMEM;
  if (!c->sw_wstat) {
    const int w = sweep_max_waves();
    if (int rc = dalloc(c, &c->sw_wstat, static_cast<size_t>(w) * 4)) return rc;
    if (int rc = dalloc(c, &c->sw_wlo, static_cast<size_t>(w) + 1)) return rc;
    c->sw_wstat_waves = w;
  }
  c->last_full = false;
  c->last_engine = FSLR_ENGINE_SWEEP;
  if (int rc = ensure_grp(c)) return rc;
  SweepArgs s{};
  s.p0 = s.p1 = nullptr;
  s.grp = c->grp;
  s.rmeta = c->rmeta;
  s.rlen8 = c->rlen8;
  s.umax = c->umax;
  s.ni = 0;
  s.nq = 0;
  s.n_reads = static_cast<int>(c->n);
  s.a_begin = 0;
  s.a_end = static_cast<int>(c->n);
  s.ent = static_cast<unsigned long long*>(const_cast<void*>(entries));
  s.ent_mid = c->ent;
  s.ent_sorted = c->ent_sorted;
  s.n_ent = n;
  s.temp = c->sweep_temp;
  s.temp_bytes = c->sweep_temp_bytes;
  s.edges = c->edges;
  s.edge_iu = c->edge_iu;
  s.edge_cap = c->edge_cap;
  s.fwd = c->fwd;
  s.counters = c->counters;
  s.err = c->errw;
  s.wstat = c->sw_wstat;
  s.wstat_waves = c->sw_wstat_waves;
  s.parent = c->parent;
  HIP_TRY(c, launch_sweep_pairs(s, 3, c->stream));
  c->hooked = true;
  return FSLR_OK;
}

int fslr_components(fslr_ctx* c) {
  if (!c) return FSLR_ERR_INVALID;
  if (!c->reads_set) return fail(c, FSLR_ERR_STATE, "fslr_set_reads first");
  HIP_TRY(c, hipSetDevice(c->device));
  if (c->prof_phases) HIP_TRY(c, hipEventRecord(c->ev[4], c->stream));
  const int n = static_cast<int>(c->n);
  const bool hooked = c->hooked;                    // the sweep's pair kernel initialised and pre-hooked parent
  c->hooked = false;
  if (!hooked) HIP_TRY(c, launch_uf_init(c->parent, n, c->stream));
  if (c->edge_cap)
    HIP_TRY(c, (hooked ? launch_uf_unions : launch_uf_edges)(c->parent, c->edges, c->counters, c->edge_cap, c->errw,
                                                             c->stream));
  HIP_TRY(c, launch_uf_finalize(c->parent, n, c->stream));
  if (c->prof_phases) HIP_TRY(c, hipEventRecord(c->ev[5], c->stream));
  c->t_comp_rec = c->prof_phases;
  return FSLR_OK;
}

int fslr_run(fslr_ctx* c, const fslr_params* p) {
  int rc = fslr_build_index(c);
  if (rc) return rc;
  if ((rc = fslr_query(c, p, 0, c->n))) return rc;
  return fslr_components(c);
}

int fslr_sync(fslr_ctx* c) {
  if (!c) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FSLR_OK;
}

#ifdef FSLR_SECTION_PROF
// diagnostics of the section-timing build (not part of the C ABI): per-read timing of the last query
extern "C" int fslr_prof_read_diag(fslr_ctx* c, uint64_t* out) {
  if (!c || !out || !c->diag) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipMemcpyAsync(out, c->diag, 2 * c->n * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FSLR_OK;
}
#endif

int fslr_read_counters(fslr_ctx* c, uint64_t* out, int n) {
  if (!c || !out || n < 0) return -FSLR_ERR_INVALID;
  if (n > kNumCounters) n = kNumCounters;
  if (!c->counters || n == 0) return 0;
  if (hipSetDevice(c->device) != hipSuccess ||
      hipMemcpyAsync(out, c->counters, n * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess)
    return -fail(c, FSLR_ERR_HIP, "reading counters");
  return n;
}

int fslr_read_stats(fslr_ctx* c, fslr_query_stats* out) {
  if (!c || !out) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  unsigned long long cnt[kNumCounters] = {};
  int ew[kErrWords] = {};
  if (c->counters) {
    HIP_TRY(c, hipMemcpyAsync(cnt, c->counters, sizeof(cnt), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipMemcpyAsync(ew, c->errw, sizeof(ew), hipMemcpyDeviceToHost, c->stream));
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  std::memset(out, 0, sizeof(*out));
  out->n_edges = static_cast<int64_t>(cnt[kEdgeCount]);
  out->evaluated_pairs = static_cast<int64_t>(cnt[kEval]);
  out->jaccard_evals = static_cast<int64_t>(cnt[kJacc]);
  out->candidates = static_cast<int64_t>(cnt[kCand]);
  out->algo_bytes = static_cast<int64_t>(cnt[kAlgoBytes]);
  out->overflow_candidates = static_cast<int64_t>(cnt[kOverflow]);
  out->gather_pairs = static_cast<int64_t>(cnt[kGather]);
  out->match_entries = static_cast<int64_t>(cnt[kMatchEntries]);
  out->matched_pairs = static_cast<int64_t>(cnt[kMatchedPairs]);
  out->walked_records = static_cast<int64_t>(cnt[kWalked]);
  out->deferred = static_cast<int64_t>(cnt[kDeferCount]);
  out->deferred_capacity = c->defer_cap;
  out->edge_capacity = c->edge_cap;
  out->engine = c->last_engine;
  ew[kErrOverflow] |= ew[kErrSticky];               // a differing repeat partition stays flagged
  out->overflow_flags = ew[kErrOverflow];
  out->pair_tests = static_cast<int64_t>(cnt[kSwTests]);
  out->entry_capacity = c->ent_cap;
  if (c->last_engine == FSLR_ENGINE_SWEEP)
    out->evaluated_pairs = out->jaccard_evals = -1;   // the sweep has no seen-set (fslr_hip.h)
  out->error = ew[0];
  out->err_a = ew[1];
  out->err_b = ew[2];
  out->max_fwd = ew[3];
  out->zd_pairs = ew[kErrZdCount];
  if (ew[kErrZdCount] > 0) {
    // the first listed pair; whether the reference raises: every pair is visited when the cap does not
    // bind (max_fwd <= edge_threshold), otherwise fslr_apply_edge_cap decides (the loops that break)
    int2 first = make_int2(0, 0);
    HIP_TRY(c, hipMemcpyAsync(&first, c->errw + kErrZdList, sizeof(first), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    out->err_a = first.x;
    out->err_b = first.y;
    const bool binds = ew[3] > c->q_thr;
    if (!c->zd_host && !binds) {
      out->error = FSLR_ERR_ZERO_DIVISION;
      c->err = "division by zero";
      return FSLR_ERR_ZERO_DIVISION;
    }
    if (!c->zd_host && ew[kErrZdCount] > c->zd_cap) {
      // the cap's replay needs every pair: a longer list, and the query again
      if (int rc = alloc_errw(c, std::max(2 * c->zd_cap, ew[kErrZdCount] + (ew[kErrZdCount] >> 2)))) return rc;
      out->overflow_flags |= 64;
      return fail(c, FSLR_ERR_STATE, "ZeroDivisionError pair list overflowed; rerun the query");
    }
    if (c->zd_host && ew[kErrZdCount] > c->zd_cap) {
      // a partition / query shard: the caller decides, and needs the list only when the cap binds (a
      // rerun then fills the longer list; the replay refuses the incomplete one). The error words stay.
      int hdr[kErrZdList];
      HIP_TRY(c, hipMemcpyAsync(hdr, c->errw, sizeof(hdr), hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(c, hipStreamSynchronize(c->stream));
      if (int rc = alloc_errw(c, std::max(2 * c->zd_cap, ew[kErrZdCount] + (ew[kErrZdCount] >> 2)))) return rc;
      hdr[kErrZdCap] = c->zd_cap;
      HIP_TRY(c, hipMemcpyAsync(c->errw, hdr, sizeof(hdr), hipMemcpyHostToDevice, c->stream));
      HIP_TRY(c, hipStreamSynchronize(c->stream));
      c->zd_lost = true;
    }
  }
  if (c->zd_lost) out->overflow_flags |= 64;
  if (out->deferred > c->defer_cap) return fail(c, FSLR_ERR_STATE, "deferred list overflowed; reserve and rerun");
  if (out->n_edges > c->edge_cap) return fail(c, FSLR_ERR_STATE, "edge buffer overflowed; reserve and rerun");
  if (ew[kErrOverflow] & 4)
    return fail(c, FSLR_ERR_STATE, "sweep partner table overflowed; rerun with FSLR_ENGINE_WALK");
  if (ew[kErrOverflow] & 24) {                       // a sync-free repeat query did not fit: rerun (with a sync)
    c->sw_prev_gen = 0;
    return fail(c, FSLR_ERR_STATE, "sweep entry buffers overflowed; rerun the query");
  }
  if (ew[kErrOverflow] & 32) {                       // a repeat partition differed from the synchronous one
    c->pt_gen = 0;
    return fail(c, FSLR_ERR_STATE, "repeat partition differs from the last synchronous one; rerun it synchronously");
  }
  return FSLR_OK;
}

int fslr_get_timings(fslr_ctx* c, fslr_timings* out) {
  if (!c || !out) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  std::memset(out, 0, sizeof(*out));
  if (!c->ev_ok) return FSLR_OK;
  if (c->t_index_rec) HIP_TRY(c, hipEventElapsedTime(&out->index_ms, c->ev[0], c->ev[1]));
  if (c->t_query_rec) HIP_TRY(c, hipEventElapsedTime(&out->query_ms, c->ev[2], c->ev[3]));
  if (c->t_kernel_rec && c->n_kern > 0) {
    const int slot = static_cast<int>((c->n_kern - 1) % fslr_ctx::kKernRing);
    HIP_TRY(c, hipEventElapsedTime(&out->pair_kernel_ms, c->kev[2 * slot], c->kev[2 * slot + 1]));
  }
  if (c->t_comp_rec) HIP_TRY(c, hipEventElapsedTime(&out->components_ms, c->ev[4], c->ev[5]));
  if (c->sw_ev_rec && c->t_query_rec && c->last_engine == FSLR_ENGINE_SWEEP) {
    HIP_TRY(c, hipEventElapsedTime(&out->sweep_count_ms, c->sw_ev[0], c->sw_ev[1]));
    HIP_TRY(c, hipEventElapsedTime(&out->sweep_emit_ms, c->sw_ev[2], c->sw_ev[3]));
    HIP_TRY(c, hipEventElapsedTime(&out->sweep_sort_ms, c->sw_ev[3], c->sw_ev[4]));
    HIP_TRY(c, hipEventElapsedTime(&out->sweep_pairs_ms, c->sw_ev[4], c->ev[3]));
  }
  if (c->t_index_rec && c->t_comp_rec) HIP_TRY(c, hipEventElapsedTime(&out->total_ms, c->ev[0], c->ev[5]));
  return FSLR_OK;
}

int fslr_get_stage_kernel_times(fslr_ctx* c, int32_t stage, float* ms, int32_t n) {
  if (!c || (!ms && n > 0) || n < 0 || stage < 0 || stage > 1) return -FSLR_ERR_INVALID;
  if (!c->ev_ok) return 0;
  if (hipSetDevice(c->device) != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess)
    return -fail(c, FSLR_ERR_HIP, "sync");
  const std::vector<hipEvent_t>& ring = stage == 0 ? c->kev : c->kev2;
  const int64_t cnt = stage == 0 ? c->n_kern : c->n_kern2;
  const int64_t have = std::min<int64_t>(cnt, fslr_ctx::kKernRing);
  const int k = static_cast<int>(std::min<int64_t>(have, n));
  for (int i = 0; i < k; ++i) {
    const int slot = static_cast<int>((cnt - k + i) % fslr_ctx::kKernRing);
    if (hipEventElapsedTime(&ms[i], ring[2 * slot], ring[2 * slot + 1]) != hipSuccess)
      return -fail(c, FSLR_ERR_HIP, "hipEventElapsedTime");
  }
  return k;
}

int fslr_get_pair_kernel_times(fslr_ctx* c, float* ms, int32_t n) { return fslr_get_stage_kernel_times(c, 0, ms, n); }

int fslr_get_labels(fslr_ctx* c, int32_t* labels) {
  if (!c || (!labels && c->n)) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  int ovf = 0;
  if (c->errw) HIP_TRY(c, hipMemcpyAsync(&ovf, c->errw + kErrOverflow, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  if (c->n) HIP_TRY(c, hipMemcpyAsync(labels, c->parent, c->n * sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  if (ovf)
    return fail(c, FSLR_ERR_STATE, "the query behind these labels overflowed its edge or deferred buffer: "
                                   "reserve and rerun it");
  return FSLR_OK;
}

int fslr_get_fwd_degree(fslr_ctx* c, int32_t* fwd) {
  if (!c || (!fwd && c->n)) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  if (c->n) HIP_TRY(c, hipMemcpyAsync(fwd, c->fwd, c->n * sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return FSLR_OK;
}

int fslr_get_edges(fslr_ctx* c, int32_t* a, int32_t* b, uint16_t* iu, int64_t capacity) {
  if (!c) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  unsigned long long cnt = 0;
  if (c->counters)
    HIP_TRY(c, hipMemcpyAsync(&cnt, c->counters + kEdgeCount, sizeof(cnt), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  const int64_t ne = static_cast<int64_t>(cnt);
  if (ne > c->edge_cap) return fail(c, FSLR_ERR_STATE, "edge buffer overflowed; reserve and rerun");
  if (ne > capacity) return fail(c, FSLR_ERR_INVALID, "output capacity too small");
  if (ne == 0) return FSLR_OK;
  std::vector<int2> tmp(static_cast<size_t>(ne));
  HIP_TRY(c, hipMemcpyAsync(tmp.data(), c->edges, ne * sizeof(int2), hipMemcpyDeviceToHost, c->stream));
  if (iu) HIP_TRY(c, hipMemcpyAsync(iu, c->edge_iu, ne * sizeof(uint16_t), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  for (int64_t k = 0; k < ne; ++k) {
    if (a) a[k] = tmp[k].x;
    if (b) b[k] = tmp[k].y;
  }
  return FSLR_OK;
}

int fslr_labels_device_ptr(fslr_ctx* c, void** dptr) {
  if (!c || !dptr) return FSLR_ERR_INVALID;
  *dptr = c->parent;
  return FSLR_OK;
}

int fslr_copy_labels_device(fslr_ctx* c, int32_t* dst) {
  if (!c || (!dst && c->n)) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  if (c->n) HIP_TRY(c, hipMemcpyAsync(dst, c->parent, c->n * sizeof(int), hipMemcpyDeviceToDevice, c->stream));
  return FSLR_OK;
}

int fslr_copy_fwd_device(fslr_ctx* c, int32_t* dst) {
  if (!c || (!dst && c->n)) return FSLR_ERR_INVALID;
  HIP_TRY(c, hipSetDevice(c->device));
  if (c->n) HIP_TRY(c, hipMemcpyAsync(dst, c->fwd, c->n * sizeof(int), hipMemcpyDeviceToDevice, c->stream));
  return FSLR_OK;
}

int fslr_union_pairs(fslr_ctx* c, const int32_t* src, const int32_t* dst, int64_t n, int on_device) {
  if (!c || !dst || n < 0) return FSLR_ERR_INVALID;
  c->hooked = false;
  HIP_TRY(c, hipSetDevice(c->device));
  if (n == 0) return FSLR_OK;
  const int* ds = src;
  const int* dd = dst;
  int* tmp = nullptr;
  if (!on_device) {
    HIP_TRY(c, hipMallocAsync(reinterpret_cast<void**>(&tmp), (src ? 2 : 1) * n * sizeof(int), c->stream));
    HIP_TRY(c, hipMemcpyAsync(tmp, dst, n * sizeof(int), hipMemcpyHostToDevice, c->stream));
    dd = tmp;
    if (src) {
      HIP_TRY(c, hipMemcpyAsync(tmp + n, src, n * sizeof(int), hipMemcpyHostToDevice, c->stream));
      ds = tmp + n;
    }
  }
  if (!src && !c->n) return fail(c, FSLR_ERR_INVALID, "no reads");
  HIP_TRY(c, launch_uf_pairs(c->parent, ds, dd, n, static_cast<int>(c->n), c->stream));
  if (tmp) {
    HIP_TRY(c, hipFreeAsync(tmp, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
  }
  return FSLR_OK;
}

int fslr_copy_edges_device(fslr_ctx* c, int32_t* dst, int64_t n_pad) {
  if (!c || (!dst && n_pad) || n_pad < 0) return FSLR_ERR_INVALID;
  if (!c->reads_set) return fail(c, FSLR_ERR_STATE, "fslr_set_reads first");
  HIP_TRY(c, hipSetDevice(c->device));
  if (n_pad == 0) return FSLR_OK;
  if (!c->edge_cap) return fail(c, FSLR_ERR_STATE, "no query has run");
  HIP_TRY(c, launch_copy_edges(c->edges, &c->counters[kEdgeCount], c->edge_cap, reinterpret_cast<int2*>(dst), n_pad,
                               c->stream));
  return FSLR_OK;
}

int fslr_local_forest(fslr_ctx* c, int64_t* n_pairs) {
  if (!c) return FSLR_ERR_INVALID;
  if (!c->reads_set) return fail(c, FSLR_ERR_STATE, "fslr_set_reads first");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const int nr = static_cast<int>(c->n);
  const bool hooked = c->hooked;                    // as in fslr_components
  c->hooked = false;
  if (!hooked) HIP_TRY(c, launch_uf_init(c->parent, nr, s));
  if (c->edge_cap)
    HIP_TRY(c, (hooked ? launch_uf_unions : launch_uf_edges)(c->parent, c->edges, c->counters, c->edge_cap, c->errw, s));
  HIP_TRY(c, launch_forest_pairs(c->parent, nr, c->forest, c->forest_cnt, c->forest_blk, s));   // finalizes too
  if (n_pairs) {
    unsigned long long k = 0;
    HIP_TRY(c, hipMemcpyAsync(&k, c->forest_cnt, sizeof(k), hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    *n_pairs = static_cast<int64_t>(k);
  }
  return FSLR_OK;
}

int fslr_copy_forest_pairs(fslr_ctx* c, int32_t* dst, int64_t n_pad) {
  if (!c || (!dst && n_pad) || n_pad < 0) return FSLR_ERR_INVALID;
  if (!c->forest || !c->forest_cnt) return fail(c, FSLR_ERR_STATE, "fslr_set_reads first");
  HIP_TRY(c, hipSetDevice(c->device));
  if (n_pad == 0) return FSLR_OK;
  HIP_TRY(c, launch_copy_edges(c->forest, c->forest_cnt, c->n, reinterpret_cast<int2*>(dst), n_pad, c->stream));
  return FSLR_OK;
}

int fslr_components_from_pairs(fslr_ctx* c, const int32_t* pairs, int64_t n) {
  if (!c || (!pairs && n) || n < 0) return FSLR_ERR_INVALID;
  c->hooked = false;
  if (!c->reads_set) return fail(c, FSLR_ERR_STATE, "fslr_set_reads first");
  HIP_TRY(c, hipSetDevice(c->device));
  const int nr = static_cast<int>(c->n);
  HIP_TRY(c, launch_uf_init(c->parent, nr, c->stream));
  HIP_TRY(c, launch_uf_pair_list(c->parent, reinterpret_cast<const int2*>(pairs), n, c->stream));
  HIP_TRY(c, launch_uf_finalize(c->parent, nr, c->stream));
  return FSLR_OK;
}

int fslr_finalize_labels(fslr_ctx* c) {
  if (!c) return FSLR_ERR_INVALID;
  c->hooked = false;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, launch_uf_finalize(c->parent, static_cast<int>(c->n), c->stream));
  return FSLR_OK;
}

}  // extern "C"
