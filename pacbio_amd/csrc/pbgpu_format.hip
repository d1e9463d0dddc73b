// pbgpu_format.hip -- the coords text of a batch, formatted on the device.
//
// print_coords (jf_aligner.cc:41-70) at GPU rates: on C2 a 50k-read step
// yields 28 M records and 4.0 GB of text, which snprintf on the host formats
// at ~1 us a record.  Here the records never leave HBM as binary:
//   k_fmt_len    one thread per record: its line length (CountSink), and per
//                read the length of its compact ">n name" header line;
//   scans        exclusive sums of both (launch_excl_scan, hand-written) -> every
//                line's byte offset;
//   k_fmt_write  one thread per record / read header: the line itself
//                (ByteSink: dword stores inside the line, bytes at its ends).
// The text is then one contiguous device buffer the driver copies to pinned
// host memory and writes.  The formatting code (pbgpu_fmt.h) is shared with
// the host test entry point pbgpu_format_double, which the CPU tests check
// against glibc's printf("%.6g").
#include <hip/hip_runtime.h>

#include "pbgpu_fmt.h"
#include "pbgpu_host.h"

namespace pbgpu {

struct FmtArgs {
  const Rec* recs;            // sorted per read (recs_sorted)
  uint32_t nrec;
  const uint64_t* rec_off;    // n_reads + 1
  uint32_t n_reads;
  const uint64_t* read_off;   // n_reads + 1 base offsets (pb_size)
  const char* pb_names;       // read names (up to the first whitespace), concatenated
  const uint64_t* pb_name_off;
  const char* sr_fwd;
  const uint64_t* sr_fwd_off;
  const char* sr_bwd;
  const uint64_t* sr_bwd_off;
  const int32_t* km;
  const int32_t* kb;
  int compact, zero_match;
};

template <class S>
__device__ inline void fmt_record(S& s, const FmtArgs& A, uint32_t i) {
  const Rec R = A.recs[i];
  const uint32_t r = R.read;
  const uint64_t n0 = A.pb_name_off[r], n1 = A.pb_name_off[r + 1];
  const bool bwd = (R.flags & 2u) != 0;
  const uint64_t* qo = bwd ? A.sr_bwd_off : A.sr_fwd_off;
  const char* qs = bwd ? A.sr_bwd : A.sr_fwd;
  const uint64_t q0 = qo[R.sr], q1 = qo[R.sr + 1];
  put_record(s, R, A.read_off[r + 1] - A.read_off[r], A.pb_names + n0, (uint32_t)(n1 - n0), A.compact != 0,
             qs + q0, (uint32_t)(q1 - q0), A.km + R.info_off, A.kb + R.info_off);
}

__device__ inline bool has_header(const FmtArgs& A, uint32_t r, uint64_t& cnt) {
  cnt = A.rec_off[r + 1] - A.rec_off[r];
  return A.compact && (cnt > 0 || A.zero_match);
}

__global__ __launch_bounds__(256) void k_fmt_len(FmtArgs A, uint32_t* rec_len, uint32_t* hdr_len) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < A.nrec) {
    CountSink c;
    fmt_record(c, A, i);
    rec_len[i] = (uint32_t)c.n;
  }
  if (i < A.n_reads) {
    uint64_t cnt;
    uint32_t L = 0;
    if (has_header(A, i, cnt)) {
      CountSink c;
      put_read_header(c, cnt, nullptr, (uint32_t)(A.pb_name_off[i + 1] - A.pb_name_off[i]));
      L = (uint32_t)c.n;
    }
    hdr_len[i] = L;
  }
}

// rec_pos / hdr_pos: exclusive scans (nrec + 1 / n_reads + 1 entries)
__global__ __launch_bounds__(256) void k_fmt_write(FmtArgs A, const uint64_t* rec_pos, const uint64_t* hdr_pos,
                                                   char* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < A.nrec) {
    const uint32_t r = A.recs[i].read;
    ByteSink s(out + hdr_pos[r + 1] + rec_pos[i]);
    fmt_record(s, A, i);
    s.finish();
  }
  if (i < A.n_reads) {
    uint64_t cnt;
    if (has_header(A, i, cnt)) {
      ByteSink s(out + hdr_pos[i] + rec_pos[A.rec_off[i]]);
      const uint64_t n0 = A.pb_name_off[i], n1 = A.pb_name_off[i + 1];
      put_read_header(s, cnt, A.pb_names + n0, (uint32_t)(n1 - n0));
      s.finish();
    }
  }
}

}  // namespace pbgpu

// super-read names (fwd and reversed) on the index's device, uploaded once
static void ensure_device_names(const pbgpu_index* cix) {
  pbgpu_index* ix = const_cast<pbgpu_index*>(cix);  // lazily built cache; guarded by names_mu
  std::lock_guard<std::mutex> lk(ix->names_mu);
  if (ix->names_ready) return;
  auto up = [&](const NameTable& v, dbuf<char>& blob, dbuf<uint64_t>& off) {
    // names of this device's super-reads (local ids [sr_begin, sr_end))
    std::vector<uint64_t> o(ix->sr_end - ix->sr_begin + 1, 0);
    for (uint64_t i = ix->sr_begin; i < ix->sr_end; ++i) o[i - ix->sr_begin + 1] = o[i - ix->sr_begin] + v[i].size();
    std::string b;
    b.reserve(o.back());
    for (uint64_t i = ix->sr_begin; i < ix->sr_end; ++i) b += v[i];
    blob.alloc(b.size() + 1);
    HIPCHK(hipMemcpy(blob.p, b.data(), b.size(), hipMemcpyHostToDevice));
    off.alloc(o.size());
    HIPCHK(hipMemcpy(off.p, o.data(), o.size() * 8, hipMemcpyHostToDevice));
  };
  HIPCHK(hipSetDevice(ix->device));
  up(ix->name_fwd, ix->d_name_fwd, ix->d_name_fwd_off);
  up(ix->name_bwd, ix->d_name_bwd, ix->d_name_bwd_off);
  ix->names_ready = true;
}

// Formats the last alignment's records (al->recs_sorted / rec_off) into
// al->text on the aligner's stream; returns the text length (synchronizes).
uint64_t format_device_text(pbgpu_aligner* al, const pbgpu_reads* rd, int compact, int zero_match) {
  const pbgpu_index* ix = al->ix;
  if (!al->have_result) throw std::invalid_argument("no result to format");
  if (ix->n_shards > 1) throw unsupported("device formatting needs a whole index (merge shard records on the host)");
  if (!rd->has_names) throw std::invalid_argument("the read batch was uploaded without read names");
  if (rd->n_reads != al->last_reads) throw std::invalid_argument("reads do not match the last alignment");
  ensure_device_names(ix);
  hipStream_t st = al->st;
  const uint32_t n = (uint32_t)al->last_reads;
  const uint64_t nrec = al->last_records;
  if (nrec > 0xFFFFFFF0ull) throw unsupported("more than 2^32 records in one batch");
  FmtArgs A;
  A.recs = al->recs_sorted.p; A.nrec = (uint32_t)nrec;
  A.rec_off = al->rec_off.p; A.n_reads = n;
  A.read_off = rd->off.p;
  A.pb_names = rd->names.p; A.pb_name_off = rd->name_off.p;
  A.sr_fwd = ix->d_name_fwd.p; A.sr_fwd_off = ix->d_name_fwd_off.p;
  A.sr_bwd = ix->d_name_bwd.p; A.sr_bwd_off = ix->d_name_bwd_off.p;
  A.km = al->info_m.p; A.kb = al->info_b.p;
  A.compact = compact; A.zero_match = zero_match;
  al->fmt_len.ensure(nrec + n + 2);
  al->fmt_pos.ensure(nrec + n + 4);
  uint32_t* rec_len = al->fmt_len.p;
  uint32_t* hdr_len = al->fmt_len.p + nrec + 1;
  uint64_t* rec_pos = al->fmt_pos.p;
  uint64_t* hdr_pos = al->fmt_pos.p + nrec + 2;
  const uint64_t items = std::max<uint64_t>(nrec, n);
  const uint32_t blocks = (uint32_t)((items + 255) / 256);
  if (blocks) {
    hipLaunchKernelGGL(k_fmt_len, dim3(blocks), dim3(256), 0, st, A, rec_len, hdr_len);
    HIPCHK(hipGetLastError());
  }
  auto scan = [&](const uint32_t* len, uint64_t m, uint64_t* pos) {
    launch_excl_scan(len, nullptr, m, pos, (uint64_t*)temp_storage(al->tmp, excl_scan_scratch_words(m) * 8), st);
  };
  scan(rec_len, nrec, rec_pos);
  scan(hdr_len, n, hdr_pos);
  uint64_t tot[2];
  HIPCHK(hipMemcpyAsync(&tot[0], rec_pos + nrec, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&tot[1], hdr_pos + n, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  const uint64_t total = tot[0] + tot[1];
  al->text.ensure(total + 4);
  if (blocks) {
    hipLaunchKernelGGL(k_fmt_write, dim3(blocks), dim3(256), 0, st, A, rec_pos, hdr_pos, al->text.p);
    HIPCHK(hipGetLastError());
  }
  al->text_len = total;
  return total;
}

extern "C" {

pbgpu_status pbgpu_format_device(pbgpu_aligner* al, const pbgpu_reads* rd, int compact, int zero_match,
                                 uint64_t* text_len) {
  if (!al || !rd || !text_len) return fail(PBGPU_ERR_INVALID, "null argument");
  if (rd->owner != al) return fail(PBGPU_ERR_INVALID, "reads were uploaded for another aligner");
  API_TRY
  HIPCHK(hipSetDevice(al->device));
  *text_len = format_device_text(al, rd, compact, zero_match);
  return PBGPU_OK;
  API_CATCH
}

pbgpu_status pbgpu_text_download(pbgpu_aligner* al, void* dst, uint64_t len) {
  if (!al || (!dst && len)) return fail(PBGPU_ERR_INVALID, "null argument");
  if (len > al->text_len) return fail(PBGPU_ERR_INVALID, "the text holds %llu bytes", (unsigned long long)al->text_len);
  API_TRY
  HIPCHK(hipSetDevice(al->device));
  if (len) HIPCHK(hipMemcpyAsync(dst, al->text.p, len, hipMemcpyDeviceToHost, al->st));
  HIPCHK(hipStreamSynchronize(al->st));
  return PBGPU_OK;
  API_CATCH
}

// Test aid: the formatter's %.6g, run on the host (the device runs the same code).
int pbgpu_format_double(double v, char* out) {
  if (!out) return -1;
  CountSink c;
  put_g6(c, v);
  ByteSink s(out);
  put_g6(s, v);
  s.finish();
  out[c.n] = 0;
  return (int)c.n;
}

}  // extern "C"
