// pbgpu_fmt.h -- the coords text of print_coords (jf_aligner.cc:41-70),
// formatted without printf so it runs on the device (k_fmt_* in
// pbgpu_format.hip) and, for the tests, on the host.
//
// The reference prints through std::ostream: integers in decimal, doubles
// with the default flags and precision 6, which libstdc++ turns into
// printf("%.*g", 6, v).  fmt_g6 reproduces glibc's %.6g bit for bit: the
// decimal value is rounded to 6 significant digits from the EXACT binary
// value with ties to even, the exponent after rounding picks fixed or
// scientific notation, trailing zeros are stripped, "inf"/"nan" with sign.
//
// Sinks: every formatter writes through a sink with put(char); CountSink
// only counts (the measure pass), ByteSink packs bytes into aligned dwords.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace pbgpu {

struct CountSink {
  uint64_t n = 0;
  __host__ __device__ inline void put(char) { ++n; }
  __host__ __device__ inline void put_str(const char* s, uint32_t len) { (void)s; n += len; }
};

// Writes bytes at p..; bytes are gathered into 4-byte words and stored as one
// dword once a word is complete and aligned; the partial words at both ends
// of a thread's range are written byte by byte (neighbouring threads own the
// other bytes of those words).
struct ByteSink {
  char* p;          // next byte position
  uint32_t w = 0;   // pending bytes of the current aligned word
  uint32_t fill = 0;
  __host__ __device__ explicit ByteSink(char* dst) : p(dst) { fill = (uint32_t)((uintptr_t)dst & 3u); }
  __host__ __device__ inline void put(char c) {
    const uint32_t sh = 8u * ((uint32_t)(uintptr_t)p & 3u);
    w |= (uint32_t)(uint8_t)c << sh;
    ++p;
    if (((uintptr_t)p & 3u) == 0) {
      if (fill == 0) {
        *(uint32_t*)(p - 4) = w;
      } else {  // first (partial) word of the range: only our bytes
        for (uint32_t i = fill; i < 4; ++i) *(p - 4 + i) = (char)(w >> (8 * i));
        fill = 0;
      }
      w = 0;
    }
  }
  __host__ __device__ inline void put_str(const char* s, uint32_t len) {
    for (uint32_t i = 0; i < len; ++i) put(s[i]);
  }
  // flush the trailing partial word (bytes fill..(p&3)-1 of it)
  __host__ __device__ inline void finish() {
    const uint32_t e = (uint32_t)((uintptr_t)p & 3u);
    if (e) {
      char* base = p - e;
      for (uint32_t i = fill; i < e; ++i) base[i] = (char)(w >> (8 * i));
    }
  }
};

// decimal digits of v (1 for 0)
__host__ __device__ inline uint32_t ndigits_u64(uint64_t v) {
  uint32_t n = 1;
  uint64_t p = 10;
  while (n < 20 && v >= p) { ++n; p *= 10; }
  return n;
}

template <class S>
__host__ __device__ inline void put_u64(S& s, uint64_t v) {
  if (v < 0x100000000ull) {  // 32-bit path: constant divisors become multiplies
    uint32_t x = (uint32_t)v;
    char d[10];
    int n = 0;
    do { d[n++] = (char)('0' + x % 10u); x /= 10u; } while (x);
    while (n) s.put(d[--n]);
    return;
  }
  char d[20];
  int n = 0;
  do { d[n++] = (char)('0' + v % 10u); v /= 10u; } while (v);
  while (n) s.put(d[--n]);
}

template <class S>
__host__ __device__ inline void put_i64(S& s, int64_t v) {
  if (v < 0) { s.put('-'); put_u64(s, (uint64_t)0 - (uint64_t)v); }
  else put_u64(s, (uint64_t)v);
}

// ---------------------------------------------------------------- %.6g
// Exact 6-significant-digit rounding.  fmt_digits6 returns D in [1e5, 1e6)
// and the decimal exponent X with |v| ~= D * 10^(X-5), rounded half to even
// on the exact binary value.

typedef unsigned __int128 u128;

__host__ __device__ inline uint64_t pow5_u64(uint32_t t) {  // t <= 27
  uint64_t p = 1;
  for (uint32_t i = 0; i < t; ++i) p *= 5;
  return p;
}

// a = M * 2^e2, s = 5 - Xe >= 0 (s <= 27): qf = floor(a * 10^s) and whether
// round-half-even goes up.  false if out of the 128-bit range.
__host__ __device__ inline bool scaled_pos(uint64_t M, int e2, int s, uint64_t& qf, bool& up) {
  const u128 N = (u128)M * pow5_u64((uint32_t)s);  // < 2^116
  const int sh = e2 + s;
  up = false;
  if (sh >= 0) {
    if (sh >= 64) return false;
    const u128 v = N << sh;
    if (v >> 64) return false;
    qf = (uint64_t)v;
    return true;
  }
  const int r = -sh;
  if (r >= 127) return false;
  const u128 qq = N >> r;
  const u128 rem = N - (qq << r);
  const u128 half = (u128)1 << (r - 1);
  if (qq >> 64) return false;
  qf = (uint64_t)qq;
  up = rem > half || (rem == half && (qf & 1));
  return true;
}

// a = M * 2^e2, t = Xe - 5 in [1, 27]: qf = floor(a / 10^t), rounding up?
__host__ __device__ inline bool scaled_neg(uint64_t M, int e2, int t, uint64_t& qf, bool& up) {
  const uint64_t p5 = pow5_u64((uint32_t)t);
  const int sh = e2 - t;  // a / 10^t = M * 2^sh / 5^t
  u128 num, den;
  if (sh >= 0) {
    if (sh > 74) return false;  // M << sh below 2^127
    num = (u128)M << sh;
    den = p5;
  } else {
    if (-sh > 63) return false;
    num = M;
    den = (u128)p5 << (-sh);
  }
  const u128 qq = num / den;
  const u128 rem = num - qq * den;
  if (qq >> 64) return false;
  qf = (uint64_t)qq;
  const u128 twice = rem << 1;
  up = twice > den || (twice == den && (qf & 1));
  return true;
}

// Slow, general path (values outside [1e-22, 1e33) or the 128-bit ranges):
// the exact decimal expansion of M * 2^e2 in base-1e9 limbs.
constexpr int FMT_LIMBS = 90;  // M * 5^1074 has < 770 digits; M * 2^971 < 2^1024 has 309
__host__ __device__ inline uint32_t fmt_pow10_u32(int e) {  // e in [0, 9]
  uint32_t p = 1;
  for (int i = 0; i < e; ++i) p *= 10;
  return p;
}
__host__ __device__ inline void digits6_bignum(uint64_t M, int e2, uint32_t& D, int& X) {
  uint32_t L[FMT_LIMBS];  // little-endian base-1e9 limbs
  int n = 0;
  for (uint64_t m = M; m; m /= 1000000000u) L[n++] = (uint32_t)(m % 1000000000u);
  int e10 = 0;  // value = limbs * 10^e10
  int left = e2 >= 0 ? e2 : -e2;
  if (e2 < 0) e10 = e2;  // M * 2^e2 = M * 5^-e2 * 10^e2
  while (left > 0) {
    const int c = e2 >= 0 ? (left > 29 ? 29 : left) : (left > 13 ? 13 : left);
    left -= c;
    uint64_t mul = 1;
    for (int i = 0; i < c; ++i) mul *= e2 >= 0 ? 2 : 5;
    uint64_t carry = 0;
    for (int i = 0; i < n; ++i) {
      const uint64_t v = (uint64_t)L[i] * mul + carry;
      L[i] = (uint32_t)(v % 1000000000u);
      carry = v / 1000000000u;
    }
    while (carry) { L[n++] = (uint32_t)(carry % 1000000000u); carry /= 1000000000u; }
  }
  int tdig = 1;  // digits of the top limb
  while (tdig < 9 && L[n - 1] >= fmt_pow10_u32(tdig)) ++tdig;
  const int total = tdig + 9 * (n - 1);
  uint32_t d = 0, r7 = 0;
  bool sticky = false;
  for (int i = 0; i < total; ++i) {  // digits, most significant first
    int limb, pos, width;
    if (i < tdig) { limb = n - 1; pos = i; width = tdig; }
    else { limb = n - 2 - (i - tdig) / 9; pos = (i - tdig) % 9; width = 9; }
    const uint32_t dig = (L[limb] / fmt_pow10_u32(width - 1 - pos)) % 10u;
    if (i < 6) d = d * 10 + dig;
    else if (i == 6) r7 = dig;
    else if (dig) { sticky = true; break; }
  }
  for (int i = total; i < 6; ++i) d *= 10;
  X = total - 1 + e10;
  if (r7 > 5 || (r7 == 5 && (sticky || (d & 1)))) {
    ++d;
    if (d == 1000000) { d = 100000; ++X; }
  }
  D = d;
}

// a > 0 finite: D in [1e5, 1e6) and X with a ~ D * 10^(X-5) (glibc %e rounding:
// exponent of a, round to 6 digits half-even, carry to the next exponent)
__host__ __device__ inline void fmt_digits6(double a, uint32_t& D, int& X) {
  const uint64_t bits = __builtin_bit_cast(uint64_t, a);
  const int be = (int)((bits >> 52) & 0x7FF);
  uint64_t M = bits & ((1ull << 52) - 1);
  int e2;
  if (be == 0) { e2 = -1074; } else { M |= 1ull << 52; e2 = be - 1075; }
  int msb = 63;
  while (!((M >> msb) & 1)) --msb;
  // a in [2^(msb+e2), 2^(msb+e2+1)): this estimate is floor(log10 a) or one less
  int Xe = (int)floor((double)(msb + e2) * 0.30102999566398120);
  for (int iter = 0; iter < 3; ++iter) {
    const int s = 5 - Xe;
    uint64_t qf = 0;
    bool up = false, ok;
    if (s >= 0 && s <= 27) ok = scaled_pos(M, e2, s, qf, up);
    else if (s < 0 && s >= -27) ok = scaled_neg(M, e2, -s, qf, up);
    else ok = false;
    if (!ok) break;
    if (qf >= 1000000u) { ++Xe; continue; }
    if (qf < 100000u) { --Xe; continue; }
    uint32_t d = (uint32_t)qf + (up ? 1u : 0u);
    X = Xe;
    if (d == 1000000u) { d = 100000u; ++X; }
    D = d;
    return;
  }
  digits6_bignum(M, e2, D, X);
}

// std::ostream << double at precision 6 == printf("%.6g")
template <class S>
__host__ __device__ inline void put_g6(S& s, double v) {
  const uint64_t bits = __builtin_bit_cast(uint64_t, v);
  const bool neg = (bits >> 63) != 0;
  const uint32_t be = (uint32_t)((bits >> 52) & 0x7FF);
  const uint64_t frac = bits & ((1ull << 52) - 1);
  if (neg) s.put('-');
  if (be == 0x7FF) {
    if (frac) { s.put('n'); s.put('a'); s.put('n'); }
    else { s.put('i'); s.put('n'); s.put('f'); }
    return;
  }
  if (be == 0 && frac == 0) { s.put('0'); return; }
  double a = neg ? -v : v;
  uint32_t D;
  int X;
  fmt_digits6(a, D, X);
  // the six digits, and how many survive trailing-zero stripping
  char dg[6];
  {
    uint32_t x = D;
    for (int i = 5; i >= 0; --i) { dg[i] = (char)('0' + x % 10u); x /= 10u; }
  }
  int nd = 6;
  while (nd > 1 && dg[nd - 1] == '0') --nd;
  if (X >= -4 && X < 6) {  // fixed: precision 5 - X
    if (X >= 0) {
      for (int i = 0; i <= X; ++i) s.put(dg[i]);
      if (nd > X + 1) {
        s.put('.');
        for (int i = X + 1; i < nd; ++i) s.put(dg[i]);
      }
    } else {
      s.put('0'); s.put('.');
      for (int i = 0; i < -X - 1; ++i) s.put('0');
      for (int i = 0; i < nd; ++i) s.put(dg[i]);
    }
  } else {  // scientific: d.ddddde+XX
    s.put(dg[0]);
    if (nd > 1) {
      s.put('.');
      for (int i = 1; i < nd; ++i) s.put(dg[i]);
    }
    s.put('e');
    int ex = X;
    if (ex < 0) { s.put('-'); ex = -ex; } else s.put('+');
    if (ex < 10) s.put('0');
    put_u64(s, (uint64_t)ex);
  }
}

}  // namespace pbgpu

namespace pbgpu {

// One record line of print_coords (jf_aligner.cc:49-67):
//   [pb_name ]rs re qs qe nb_mers pb_cons sr_cons pb_cover sr_cover pb_size ql
//   stretch offset avg_err qname[ k:b]...\n
// (non-compact mode prefixes the read name).  Rec is pbgpu_internal.h's.
template <class S, class R>
__host__ __device__ inline void put_record(S& s, const R& r, uint64_t pb_size, const char* pb_name, uint32_t pb_name_len,
                                           bool compact, const char* qname, uint32_t qname_len, const int32_t* km,
                                           const int32_t* kb) {
  if (!compact) { s.put_str(pb_name, pb_name_len); s.put(' '); }
  put_i64(s, r.rs); s.put(' ');
  put_i64(s, r.re); s.put(' ');
  put_i64(s, r.qs); s.put(' ');
  put_i64(s, r.qe); s.put(' ');
  put_i64(s, r.nb_mers); s.put(' ');
  put_u64(s, r.pb_cons); s.put(' ');
  put_u64(s, r.sr_cons); s.put(' ');
  put_u64(s, r.pb_cover); s.put(' ');
  put_u64(s, r.sr_cover); s.put(' ');
  put_u64(s, pb_size); s.put(' ');
  put_u64(s, r.ql); s.put(' ');
  put_g6(s, r.stretch); s.put(' ');
  put_g6(s, r.offset); s.put(' ');
  put_g6(s, r.avg_err); s.put(' ');
  s.put_str(qname, qname_len);
  for (uint32_t t = 0; t < r.n_info; ++t) {
    s.put(' ');
    put_i64(s, km[t]);
    s.put(':');
    put_i64(s, kb[t]);
  }
  s.put('\n');
}

// The compact per-read header (jf_aligner.cc:47-48): ">" n " " pb_name "\n"
template <class S>
__host__ __device__ inline void put_read_header(S& s, uint64_t n, const char* pb_name, uint32_t pb_name_len) {
  s.put('>');
  put_u64(s, n);
  s.put(' ');
  s.put_str(pb_name, pb_name_len);
  s.put('\n');
}

}  // namespace pbgpu
