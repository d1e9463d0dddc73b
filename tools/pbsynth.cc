// pbsynth -- deterministic synthetic workload generator.
//
//   genome  : i.i.d. uniform ACGT (optionally with a repeat model: a fraction
//             of the genome is covered by 5-50 copies of 1-6 kb elements at
//             1% divergence, which exercises --max-count and the 99% threshold)
//   unitigs : the genome cut into lognormal segments (mean 300, min 100) that
//             overlap by K_u-1; lengths file "id len"
//   SRs     : random walks of 1-8 consecutive unitigs, named "12F_13F_14F";
//             50% emitted reverse-complemented with the reversed name
//             ("14R_13R_12R"); pure ACGT
//   PB      : uniform start, strand 50/50, fixed or lognormal length, CLR error
//             model (ins/del/sub i.i.d. per base) plus rare N runs; names 0,1,..
//
// Every SR / PB record draws from its own mt19937_64 seeded by
// splitmix64(seed, stream, index), so generation is parallel and the output is
// independent of the thread count.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

extern "C" {
struct pbsynth_config {
  uint64_t genome_len;
  uint64_t seed;
  uint64_t n_sr;
  uint64_t n_pb;
  double   pb_len_mean;    // fixed length when pb_len_sigma == 0
  double   pb_len_sigma;   // lognormal sigma
  uint32_t pb_len_min, pb_len_max;
  double   err_ins, err_del, err_sub; // per-base CLR error rates
  double   n_run_rate;     // per-base probability of starting an N run (length 1-20)
  uint32_t unitig_k;       // K_u (unitigs overlap by K_u-1)
  double   unitig_mean;
  uint32_t unitig_min;
  uint32_t sr_max_unitigs; // random walk length in [1, sr_max_unitigs]
  double   repeat_frac;    // fraction of the genome covered by repeat copies (0 = none)
  uint64_t pb_index_base;  // PB read i is drawn as global read pb_index_base + i (rank shards)
};

struct pbsynth_seqs {
  uint64_t  n;
  char*     seq;       // concatenated sequences
  uint64_t* off;       // n+1 offsets into seq
  char*     names;     // concatenated NUL-terminated names
  uint64_t* name_off;  // n offsets into names
};
}

namespace {
inline uint64_t splitmix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ULL;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
  return x ^ (x >> 31);
}
inline uint64_t stream_seed(uint64_t seed, uint64_t stream, uint64_t idx) {
  return splitmix64(splitmix64(seed ^ (stream * 0x632be59bd9b4e019ULL)) + idx);
}
const char BASES[4] = {'A', 'C', 'G', 'T'};
inline char comp(char c) {
  switch (c) { case 'A': return 'T'; case 'C': return 'G'; case 'G': return 'C'; case 'T': return 'A'; default: return 'N'; }
}

template <typename F>
void parallel_for(uint64_t n, int threads, F f) {
  if (threads < 1) threads = 1;
  std::atomic<uint64_t> next(0);
  const uint64_t chunk = 64;
  auto work = [&]() {
    for (;;) {
      uint64_t s = next.fetch_add(chunk);
      if (s >= n) break;
      uint64_t e = std::min(n, s + chunk);
      for (uint64_t i = s; i < e; ++i) f(i);
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < threads; ++t) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
}

struct gen_state {
  std::string genome;
  std::vector<uint64_t> ustart, ulen;
};

void make_genome(const pbsynth_config& c, int threads, gen_state& g) {
  g.genome.assign(c.genome_len, 'A');
  const uint64_t block = 1 << 20;
  const uint64_t nb = (c.genome_len + block - 1) / block;
  parallel_for(nb, threads, [&](uint64_t b) {
    std::mt19937_64 r(stream_seed(c.seed, 1, b));
    uint64_t s = b * block, e = std::min(c.genome_len, s + block);
    for (uint64_t i = s; i < e; ++i) g.genome[i] = BASES[r() & 3];
  });
  if (c.repeat_frac > 0) {
    // Repeat model: elements of 1-6 kb, each copied 5-50 times with 1%
    // substitutions, pasted at uniform positions until repeat_frac of the
    // genome is covered (sequential: deterministic overlap order).
    std::mt19937_64 r(stream_seed(c.seed, 2, 0));
    uint64_t covered = 0, target = (uint64_t)(c.repeat_frac * (double)c.genome_len);
    while (covered < target && c.genome_len > 10000) {
      uint64_t len = 1000 + r() % 5001;
      uint64_t src = r() % (c.genome_len - len);
      std::string elem = g.genome.substr(src, len);
      uint64_t copies = 5 + r() % 46;
      for (uint64_t k = 0; k < copies; ++k) {
        uint64_t dst = r() % (c.genome_len - len);
        for (uint64_t i = 0; i < len; ++i) {
          char b = elem[i];
          if ((r() % 100) == 0) b = BASES[r() & 3];
          g.genome[dst + i] = b;
        }
        covered += len;
      }
    }
  }
}

void make_unitigs(const pbsynth_config& c, gen_state& g) {
  std::mt19937_64 r(stream_seed(c.seed, 3, 0));
  const double sigma = 0.5, mu = std::log(c.unitig_mean) - sigma * sigma / 2;
  std::lognormal_distribution<double> ln(mu, sigma);
  const uint64_t ov = c.unitig_k - 1;
  uint64_t s = 0;
  while (true) {
    uint64_t len = std::max<uint64_t>(c.unitig_min, (uint64_t)ln(r));
    if (len <= ov) len = ov + 1;
    if (s + len >= c.genome_len) { len = c.genome_len - s; g.ustart.push_back(s); g.ulen.push_back(len); break; }
    g.ustart.push_back(s); g.ulen.push_back(len);
    s += len - ov;
  }
}

void pack(std::vector<std::string>& seqs, std::vector<std::string>& names, pbsynth_seqs* out) {
  uint64_t n = seqs.size(), total = 0, ntotal = 0;
  for (auto& s : seqs) total += s.size();
  for (auto& s : names) ntotal += s.size() + 1;
  out->n = n;
  out->seq = (char*)malloc(total + 1);
  out->off = (uint64_t*)malloc((n + 1) * sizeof(uint64_t));
  out->names = (char*)malloc(ntotal + 1);
  out->name_off = (uint64_t*)malloc((n + 1) * sizeof(uint64_t));
  uint64_t o = 0, no = 0;
  for (uint64_t i = 0; i < n; ++i) {
    out->off[i] = o;
    memcpy(out->seq + o, seqs[i].data(), seqs[i].size());
    o += seqs[i].size();
    std::string().swap(seqs[i]);
    out->name_off[i] = no;
    memcpy(out->names + no, names[i].c_str(), names[i].size() + 1);
    no += names[i].size() + 1;
  }
  out->off[n] = o;
  out->seq[o] = 0;
}
}  // namespace

extern "C" {
void pbsynth_default(pbsynth_config* c) {
  memset(c, 0, sizeof(*c));
  c->genome_len = 1000000; c->seed = 42; c->n_sr = 1000; c->n_pb = 100;
  c->pb_len_mean = 10000; c->pb_len_sigma = 0; c->pb_len_min = 500; c->pb_len_max = 100000;
  c->err_ins = 0.07; c->err_del = 0.04; c->err_sub = 0.02; c->n_run_rate = 0.001 / 10;
  c->unitig_k = 31; c->unitig_mean = 300; c->unitig_min = 100; c->sr_max_unitigs = 8; c->repeat_frac = 0;
}

int pbsynth_make(const pbsynth_config* cfg, int threads, pbsynth_seqs* sr, pbsynth_seqs* pb,
                 int32_t** ul, uint64_t* n_ul) {
  const pbsynth_config& c = *cfg;
  if (c.genome_len < 1000 || c.unitig_k < 2) return 1;
  gen_state g;
  make_genome(c, threads, g);
  make_unitigs(c, g);
  const uint64_t nu = g.ustart.size();
  *n_ul = nu;
  *ul = (int32_t*)malloc(nu * sizeof(int32_t));
  for (uint64_t i = 0; i < nu; ++i) (*ul)[i] = (int32_t)g.ulen[i];

  if (sr) {
    // Two passes, written straight into the output buffers (C5: 50M SRs, ~60 Gbp):
    // pass 1 draws each SR's walk (its own RNG stream) and sizes it, pass 2 copies.
    const uint64_t n = c.n_sr;
    std::vector<uint64_t> su(n);             // first unitig
    std::vector<uint32_t> scnt(n);           // unitig count << 1 | reverse
    std::vector<uint64_t> off(n + 1, 0), noff(n + 1, 0);
    parallel_for(n, threads, [&](uint64_t i) {
      std::mt19937_64 r(stream_seed(c.seed, 4, i));
      uint64_t cnt = 1 + r() % c.sr_max_unitigs;
      uint64_t u = r() % nu;
      if (u + cnt > nu) cnt = nu - u;
      const bool rev = r() & 1;
      su[i] = u;
      scnt[i] = (uint32_t)(cnt << 1 | (rev ? 1 : 0));
      off[i + 1] = g.ustart[u + cnt - 1] + g.ulen[u + cnt - 1] - g.ustart[u];
      uint64_t nl = 0;  // "12F_13F_14F" + NUL
      for (uint64_t t = 0; t < cnt; ++t) nl += (t ? 1 : 0) + std::to_string(u + t).size() + 1;
      noff[i + 1] = nl + 1;
    });
    for (uint64_t i = 0; i < n; ++i) { off[i + 1] += off[i]; noff[i + 1] += noff[i]; }
    sr->n = n;
    sr->seq = (char*)malloc(off[n] + 1);
    sr->off = (uint64_t*)malloc((n + 1) * sizeof(uint64_t));
    sr->names = (char*)malloc(noff[n] + 1);
    sr->name_off = (uint64_t*)malloc((n + 1) * sizeof(uint64_t));
    if (!sr->seq || !sr->off || !sr->names || !sr->name_off) return 2;
    memcpy(sr->off, off.data(), (n + 1) * sizeof(uint64_t));
    memcpy(sr->name_off, noff.data(), (n + 1) * sizeof(uint64_t));
    sr->seq[off[n]] = 0;
    sr->names[noff[n]] = 0;
    parallel_for(n, threads, [&](uint64_t i) {
      const uint64_t u = su[i], cnt = scnt[i] >> 1;
      const bool rev = scnt[i] & 1;
      const uint64_t s = g.ustart[u], len = off[i + 1] - off[i];
      char* d = sr->seq + off[i];
      std::string name;
      if (!rev) {
        memcpy(d, g.genome.data() + s, len);
        for (uint64_t t = 0; t < cnt; ++t) name += (t ? "_" : "") + std::to_string(u + t) + "F";
      } else {
        for (uint64_t t = 0; t < len; ++t) d[t] = comp(g.genome[s + len - 1 - t]);
        for (uint64_t t = 0; t < cnt; ++t) name += (t ? "_" : "") + std::to_string(u + cnt - 1 - t) + "R";
      }
      memcpy(sr->names + noff[i], name.c_str(), name.size() + 1);
    });
  }
  if (pb) {
    std::vector<std::string> seqs(c.n_pb), names(c.n_pb);
    const double psig = c.pb_len_sigma, pmu = std::log(c.pb_len_mean) - psig * psig / 2;
    parallel_for(c.n_pb, threads, [&](uint64_t i) {
      std::mt19937_64 r(stream_seed(c.seed, 5, c.pb_index_base + i));
      uint64_t len = (uint64_t)c.pb_len_mean;
      if (psig > 0) {
        std::lognormal_distribution<double> ln(pmu, psig);
        len = (uint64_t)ln(r);
        len = std::min<uint64_t>(std::max<uint64_t>(len, c.pb_len_min), c.pb_len_max);
      }
      len = std::min<uint64_t>(len, c.genome_len);
      uint64_t s = r() % (c.genome_len - len + 1);
      std::string tmpl = g.genome.substr(s, len);
      if (r() & 1) { std::reverse(tmpl.begin(), tmpl.end()); for (auto& ch : tmpl) ch = comp(ch); }
      std::string out;
      out.reserve(len + len / 8);
      std::uniform_real_distribution<double> U(0.0, 1.0);
      const double pi = c.err_ins, pd = pi + c.err_del, ps = pd + c.err_sub;
      for (uint64_t t = 0; t < len; ++t) {
        double x = U(r);
        if (x < pi) { out.push_back(BASES[r() & 3]); out.push_back(tmpl[t]); }
        else if (x < pd) { /* deletion */ }
        else if (x < ps) { char b; do { b = BASES[r() & 3]; } while (b == tmpl[t]); out.push_back(b); }
        else out.push_back(tmpl[t]);
        if (c.n_run_rate > 0 && U(r) < c.n_run_rate) { uint64_t nl = 1 + r() % 20; out.append(nl, 'N'); }
      }
      seqs[i].swap(out);
      names[i] = std::to_string(c.pb_index_base + i);
    });
    pack(seqs, names, pb);
  }
  return 0;
}

void pbsynth_free(pbsynth_seqs* s) {
  if (!s) return;
  free(s->seq); free(s->off); free(s->names); free(s->name_off);
  memset(s, 0, sizeof(*s));
}
void pbsynth_free_ul(int32_t* ul) { free(ul); }

int pbsynth_write_fasta(const pbsynth_seqs* s, const char* path, int line_width) {
  FILE* f = fopen(path, "w");
  if (!f) return 1;
  for (uint64_t i = 0; i < s->n; ++i) {
    fprintf(f, ">%s\n", s->names + s->name_off[i]);
    uint64_t a = s->off[i], b = s->off[i + 1];
    if (line_width <= 0) { fwrite(s->seq + a, 1, b - a, f); fputc('\n', f); }
    else for (uint64_t p = a; p < b; p += (uint64_t)line_width) {
      uint64_t e = std::min(b, p + (uint64_t)line_width);
      fwrite(s->seq + p, 1, e - p, f); fputc('\n', f);
    }
  }
  return fclose(f);
}

int pbsynth_write_ul(const int32_t* ul, uint64_t n, const char* path) {
  FILE* f = fopen(path, "w");
  if (!f) return 1;
  for (uint64_t i = 0; i < n; ++i) fprintf(f, "%llu %d\n", (unsigned long long)i, ul[i]);
  return fclose(f);
}
}

#ifdef PBSYNTH_MAIN
// CLI: pbsynth <preset C1|C2|C3|tiny> <outdir> [seed] [n_pb override]
int main(int argc, char** argv) {
  if (argc < 3) { fprintf(stderr, "usage: pbsynth C1|C2|C3|tiny outdir [seed] [n_pb]\n"); return 1; }
  pbsynth_config c; pbsynth_default(&c);
  std::string p = argv[1];
  if (p == "C1") { c.genome_len = 1000000; c.n_sr = 1000; c.n_pb = 100; c.pb_len_mean = 10000; }
  else if (p == "C2") { c.genome_len = 4600000; c.n_sr = 200000; c.n_pb = 50000; c.pb_len_mean = 12000; c.pb_len_sigma = 0.5; }
  else if (p == "C3") { c.genome_len = 12000000; c.n_sr = 1000000; c.n_pb = 300000; c.pb_len_mean = 12000; c.pb_len_sigma = 0.5; }
  else if (p == "tiny") { c.genome_len = 20000; c.n_sr = 60; c.n_pb = 8; c.pb_len_mean = 2000; }
  else { fprintf(stderr, "unknown preset\n"); return 1; }
  if (argc > 3) c.seed = strtoull(argv[3], nullptr, 10);
  if (argc > 4) c.n_pb = strtoull(argv[4], nullptr, 10);
  pbsynth_seqs sr, pb; int32_t* ul; uint64_t nul;
  if (pbsynth_make(&c, (int)std::thread::hardware_concurrency(), &sr, &pb, &ul, &nul)) return 1;
  std::string d = argv[2];
  pbsynth_write_fasta(&sr, (d + "/sr.fa").c_str(), 70);
  pbsynth_write_fasta(&pb, (d + "/pb.fa").c_str(), 0);
  pbsynth_write_ul(ul, nul, (d + "/ul.txt").c_str());
  return 0;
}
#endif
