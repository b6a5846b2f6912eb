/*
 * zfp_oracle.c -- TEST INFRASTRUCTURE ONLY. Not part of the product; never linked by libgcow.so.
 *
 * Clean-room CPU restatement of the gcow sw/ block codec, written from the per-block spec
 * (SURVEY.md Appendix A), each function citing the reference file:line it restates.
 * Extended from sw/'s 2-D-only driver to d = 1, 2, 3 following LLNL zfp 0.5.5 (which sw/ is
 * byte-identical to on 2-D); the 1-D/3-D/decode behaviour is pinned by libzfp-generated fixtures.
 * Callers: tests/, __graft_entry__.smoke(), bench.py cpu_baseline.
 */
#include "zfp_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define EBITS 8
#define EBIAS 127
#define NBMASK 0xaaaaaaaau
#define OMIN(a, b) ((a) < (b) ? (a) : (b))
#define OMAX(a, b) ((a) > (b) ? (a) : (b))

/* ------------------------------------------------------------------------------------------------
 * Bit I/O: LSB-first into little-endian uint64 words (sw/src/stream.c:61-138). Output words must
 * be zero-initialised; bits are OR-ed in at absolute bit offsets.
 * ---------------------------------------------------------------------------------------------- */
static inline void put_bits(uint64_t* w, uint64_t* pos, uint64_t v, unsigned n)
{
  if (!n) return;
  if (n < 64) v &= ((uint64_t)1 << n) - 1;
  uint64_t p = *pos;
  unsigned sh = (unsigned)(p & 63);
  w[p >> 6] |= v << sh;
  if (sh && sh + n > 64) w[(p >> 6) + 1] |= v >> (64 - sh);
  *pos = p + n;
}

static inline unsigned put_bit(uint64_t* w, uint64_t* pos, unsigned bit)
{
  if (bit) w[*pos >> 6] |= (uint64_t)1 << (*pos & 63);
  (*pos)++;
  return bit;
}

static inline uint64_t get_bits(const uint64_t* w, uint64_t* pos, unsigned n)
{
  if (!n) return 0;
  uint64_t p = *pos;
  unsigned sh = (unsigned)(p & 63);
  uint64_t v = w[p >> 6] >> sh;
  if (sh && sh + n > 64) v |= w[(p >> 6) + 1] << (64 - sh);
  if (n < 64) v &= ((uint64_t)1 << n) - 1;
  *pos = p + n;
  return v;
}

static inline unsigned get_bit(const uint64_t* w, uint64_t* pos)
{
  unsigned b = (unsigned)(w[*pos >> 6] >> (*pos & 63)) & 1u;
  (*pos)++;
  return b;
}

/* ------------------------------------------------------------------------------------------------
 * Parameters (sw/src/common.c:6-21, 226-236)
 * ---------------------------------------------------------------------------------------------- */
unsigned orc_precision(int emax, unsigned maxprec, int minexp, unsigned dims)
{
  /* common.c:226-229 */
  int p = emax - minexp + 2 * (int)dims + 2;
  return OMIN(maxprec, (unsigned)OMAX(0, p));
}

static int exceeded_maxbits(unsigned maxbits, unsigned maxprec, unsigned size)
{
  /* common.c:232-236 */
  return (maxprec + 1) * size - 1 > maxbits;
}

void orc_set_accuracy(orc_params* p, double tol)
{
  /* common.c:6-21 */
  int emin = -1074;
  if (tol > 0) {
    frexp(tol, &emin);
    emin--;
  }
  p->minbits = 1;
  p->maxbits = 16658; /* sw/include/common.h:11 (libzfp 16657; identical for d <= 3) */
  p->maxprec = 64;
  p->minexp = emin;
}

void orc_set_rate(orc_params* p, double rate, unsigned dims)
{
  /* libzfp 0.5.5 zfp_stream_set_rate (non-wra), float: bits = max(floor(4^d rate + 0.5), 1 + 8) */
  unsigned n = 1u << (2 * dims);
  unsigned bits = (unsigned)floor(n * rate + 0.5);
  if (bits < 9) bits = 9;
  p->minbits = bits;
  p->maxbits = bits;
  p->maxprec = 64;
  p->minexp = -1074;
}

void orc_set_precision(orc_params* p, unsigned prec)
{
  /* libzfp 0.5.5 zfp_stream_set_precision */
  p->minbits = 1;
  p->maxbits = 16658;
  p->maxprec = prec ? OMIN(prec, 64u) : 64u;
  p->minexp = -1074;
}

/* ------------------------------------------------------------------------------------------------
 * Stages (sw/src/encode.c)
 * ---------------------------------------------------------------------------------------------- */
int orc_block_exponent(const float* block, unsigned n)
{
  /* encode.c:142-152 + get_scaler_exponent :128-140. NaN never wins `max < f`; glibc frexp(inf) -> 0. */
  float max = 0;
  do {
    float f = fabsf(*block++);
    if (max < f) max = f;
  } while (--n);
  int e = -EBIAS;
  if (max > 0) {
    frexp((double)max, &e);
    e = OMAX(e, 1 - EBIAS);
  }
  return e;
}

void orc_fwd_cast(int32_t* iblock, const float* fblock, unsigned n, int emax)
{
  /* encode.c:162-187. scale = 2^(30-emax) (+inf when emax <= -98). x86 (int32) of NaN / out-of-range gives
   * INT_MIN (cvttss2si "integer indefinite"); stated explicitly here so the oracle has no UB. */
  float scale = (float)ldexp(1.0, 30 - emax);
  do {
    float p = scale * *fblock++;
    *iblock++ = (fabsf(p) < 2147483648.0f) ? (int32_t)p : INT32_MIN;
  } while (--n);
}

static inline int32_t wadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
static inline int32_t wsub(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }
static inline int32_t wshl1(int32_t a) { return (int32_t)((uint32_t)a << 1); }

static void fwd_lift(int32_t* p, ptrdiff_t s)
{
  /* encode.c:189-249 with int32 wraparound made explicit */
  int32_t x = p[0], y = p[s], z = p[2 * s], w = p[3 * s];
  x = wadd(x, w); x >>= 1; w = wsub(w, x);
  z = wadd(z, y); z >>= 1; y = wsub(y, z);
  x = wadd(x, z); x >>= 1; z = wsub(z, x);
  w = wadd(w, y); w >>= 1; y = wsub(y, w);
  w = wadd(w, y >> 1); y = wsub(y, w >> 1);
  p[0] = x; p[s] = y; p[2 * s] = z; p[3 * s] = w;
}

static void inv_lift(int32_t* p, ptrdiff_t s)
{
  /* decode.c:58-100 */
  int32_t x = p[0], y = p[s], z = p[2 * s], w = p[3 * s];
  y = wadd(y, w >> 1); w = wsub(w, y >> 1);
  y = wadd(y, w); w = wshl1(w); w = wsub(w, y);
  z = wadd(z, x); x = wshl1(x); x = wsub(x, z);
  y = wadd(y, z); z = wshl1(z); z = wsub(z, y);
  w = wadd(w, x); x = wshl1(x); x = wsub(x, w);
  p[0] = x; p[s] = y; p[2 * s] = z; p[3 * s] = w;
}

void orc_fwd_xform(int32_t* q, unsigned dims)
{
  /* encode.c:251-260 (2-D: x then y); 1-D one lift; 3-D x, y, z as libzfp */
  unsigned x, y, z;
  switch (dims) {
    case 1:
      fwd_lift(q, 1);
      break;
    case 2:
      for (y = 0; y < 4; y++) fwd_lift(q + 4 * y, 1);
      for (x = 0; x < 4; x++) fwd_lift(q + x, 4);
      break;
    case 3:
      for (z = 0; z < 4; z++)
        for (y = 0; y < 4; y++) fwd_lift(q + 4 * y + 16 * z, 1);
      for (x = 0; x < 4; x++)
        for (z = 0; z < 4; z++) fwd_lift(q + 16 * z + x, 4);
      for (y = 0; y < 4; y++)
        for (x = 0; x < 4; x++) fwd_lift(q + x + 4 * y, 16);
      break;
    case 4: /* libzfp 0.5.5 fwd_xform_4: x, y, z, then w */
      for (unsigned l = 0; l < 64; l++) fwd_lift(q + 4 * l, 1);
      for (unsigned l = 0; l < 64; l++) fwd_lift(q + (l & 3) + 16 * (l >> 2), 4);
      for (unsigned l = 0; l < 64; l++) fwd_lift(q + (l & 15) + 64 * (l >> 4), 16);
      for (unsigned l = 0; l < 64; l++) fwd_lift(q + l, 64);
      break;
  }
}

void orc_inv_xform(int32_t* q, unsigned dims)
{
  /* decode.c:102-111 (2-D: y then x); 3-D z, y, x */
  unsigned x, y, z;
  switch (dims) {
    case 1:
      inv_lift(q, 1);
      break;
    case 2:
      for (x = 0; x < 4; x++) inv_lift(q + x, 4);
      for (y = 0; y < 4; y++) inv_lift(q + 4 * y, 1);
      break;
    case 3:
      for (y = 0; y < 4; y++)
        for (x = 0; x < 4; x++) inv_lift(q + x + 4 * y, 16);
      for (x = 0; x < 4; x++)
        for (z = 0; z < 4; z++) inv_lift(q + 16 * z + x, 4);
      for (z = 0; z < 4; z++)
        for (y = 0; y < 4; y++) inv_lift(q + 4 * y + 16 * z, 1);
      break;
    case 4: /* w, z, y, then x */
      for (unsigned l = 0; l < 64; l++) inv_lift(q + l, 64);
      for (unsigned l = 0; l < 64; l++) inv_lift(q + (l & 15) + 64 * (l >> 4), 16);
      for (unsigned l = 0; l < 64; l++) inv_lift(q + (l & 3) + 16 * (l >> 2), 4);
      for (unsigned l = 0; l < 64; l++) inv_lift(q + 4 * l, 1);
      break;
  }
}

static const unsigned char PERM1[4] = {0, 1, 2, 3};
/* sw/include/types.h:71-97 */
static const unsigned char PERM2[16] = {0, 1, 4, 5, 2, 8, 6, 9, 3, 12, 10, 7, 13, 11, 14, 15};
/* libzfp 0.5.5 perm_3 (ordered by i+j+k, then i^2+j^2+k^2); SURVEY 8(a) A11 */
static const unsigned char PERM3[64] = {
    0,  1,  4,  16, 20, 17, 5,  2,  8,  32, 21, 6,  18, 24, 9,  33, 36, 3,  12, 48, 22, 25,
    37, 40, 34, 10, 7,  19, 28, 13, 49, 52, 41, 38, 26, 23, 29, 53, 11, 35, 44, 14, 50, 56,
    42, 27, 39, 45, 30, 54, 57, 60, 51, 15, 43, 46, 58, 61, 55, 31, 62, 59, 47, 63};

/* libzfp 0.5.5 perm_4 (rodata of /opt/conda/lib/libzfp.so.0.5.5 at 0x4ca00), pinned by the
 * 4-D libzfp fixtures */
static const unsigned char PERM4[256] = {
    0,   1,   4,   16,  64,  5,   80,  17,  68,  65,  20,  2,   8,   32,  128, 84,  81,  69,  21,  6,   18,  66,
    24,  72,  9,   96,  33,  36,  129, 132, 144, 3,   12,  48,  192, 85,  82,  70,  22,  73,  25,  88,  37,  100,
    97,  148, 145, 133, 10,  160, 34,  136, 130, 40,  7,   19,  67,  28,  76,  13,  112, 49,  52,  193, 196, 208,
    86,  89,  101, 149, 161, 137, 41,  134, 38,  164, 26,  152, 146, 104, 98,  74,  83,  71,  23,  77,  29,  92,
    53,  116, 113, 212, 209, 197, 11,  35,  131, 44,  140, 14,  176, 50,  56,  194, 200, 224, 90,  165, 102, 153,
    150, 105, 168, 162, 138, 42,  87,  93,  117, 213, 27,  75,  99,  39,  135, 147, 108, 45,  141, 156, 30,  78,
    177, 180, 54,  114, 120, 57,  198, 210, 216, 201, 225, 228, 15,  240, 51,  204, 195, 60,  169, 166, 154, 106,
    91,  103, 151, 109, 157, 94,  181, 118, 121, 214, 217, 229, 163, 139, 43,  142, 46,  172, 58,  184, 178, 232,
    226, 202, 241, 205, 61,  199, 55,  244, 31,  220, 211, 124, 115, 79,  170, 167, 155, 107, 158, 110, 173, 122,
    185, 182, 233, 230, 218, 95,  245, 119, 221, 215, 125, 242, 206, 62,  203, 59,  248, 47,  236, 227, 188, 179,
    143, 171, 174, 186, 234, 246, 222, 126, 219, 123, 249, 111, 237, 231, 189, 183, 159, 252, 243, 207, 63,  175,
    250, 187, 238, 235, 190, 253, 247, 223, 127, 254, 251, 239, 191, 255};

const unsigned char* orc_perm(unsigned dims)
{
  return dims == 1 ? PERM1 : dims == 2 ? PERM2 : dims == 3 ? PERM3 : PERM4;
}

void orc_fwd_reorder(uint32_t* u, const int32_t* q, unsigned dims)
{
  /* encode.c:263-275 (without the one-past-the-end write of :272-274) */
  const unsigned char* perm = orc_perm(dims);
  unsigned size = 1u << (2 * dims);
  for (unsigned i = 0; i < size; i++) u[i] = ((uint32_t)q[perm[i]] + NBMASK) ^ NBMASK;
}

/* 256-bit bit planes for 4-D blocks (x[0] holds coefficients 0..63) */
static uint64_t wide_bits(const uint64_t* x, unsigned o)
{
  unsigned i = o >> 6, sh = o & 63;
  uint64_t v = i < 4 ? x[i] >> sh : 0;
  if (sh && i + 1 < 4) v |= x[i + 1] << (64 - sh);
  return v;
}

static void wide_shr(uint64_t* x, unsigned m)
{
  uint64_t y[4];
  for (unsigned i = 0; i < 4; i++) y[i] = m + 64 * i < 256 ? wide_bits(x, m + 64 * i) : 0;
  memcpy(x, y, sizeof(y));
}

static int wide_nonzero(const uint64_t* x) { return (x[0] | x[1] | x[2] | x[3]) != 0; }

/* encode.c:279-339 for 256 coefficients (the same loop, planes of 256 bits) */
static unsigned encode_ints_256(uint64_t* w, uint64_t* pos, const uint32_t* u, unsigned maxbits, unsigned maxprec)
{
  unsigned intprec = 32;
  unsigned kmin = intprec > maxprec ? intprec - maxprec : 0;
  unsigned bits = maxbits;
  unsigned k, m, n;
  for (k = intprec, n = 0; bits && k-- > kmin;) {
    uint64_t x[4] = {0, 0, 0, 0};
    for (unsigned i = 0; i < 256; i++) x[i >> 6] |= (uint64_t)((u[i] >> k) & 1u) << (i & 63);
    m = OMIN(n, bits);
    bits -= m;
    for (unsigned o = 0; o < m; o += 64) put_bits(w, pos, wide_bits(x, o), OMIN(64u, m - o));
    wide_shr(x, m);
    for (; bits && n < 256; wide_shr(x, 1), n++) {
      bits--;
      if (put_bit(w, pos, (unsigned)wide_nonzero(x))) {
        for (; bits && n < 255; wide_shr(x, 1), n++) {
          bits--;
          if (put_bit(w, pos, (unsigned)(x[0] & 1u))) break;
        }
      } else {
        break;
      }
    }
  }
  return maxbits - bits;
}

unsigned orc_encode_ints(uint64_t* w, uint64_t* pos, const uint32_t* u, unsigned maxbits, unsigned maxprec,
                         unsigned size)
{
  if (size == 256) return encode_ints_256(w, pos, u, maxbits, maxprec);
  /* encode.c:279-339 (partial) == encode.c:343-408 (all) whenever the budget is not hit */
  unsigned intprec = 32;
  unsigned kmin = intprec > maxprec ? intprec - maxprec : 0;
  unsigned bits = maxbits;
  unsigned i, k, m, n;
  for (k = intprec, n = 0; bits && k-- > kmin;) {
    uint64_t x = 0;
    for (i = 0; i < size; i++) x += (uint64_t)((u[i] >> k) & 1u) << i;
    m = OMIN(n, bits);
    bits -= m;
    put_bits(w, pos, x, m);
    x = m < 64 ? x >> m : 0;
    for (; bits && n < size; x >>= 1, n++) {
      bits--;
      if (put_bit(w, pos, !!x)) {
        for (; bits && n < size - 1; x >>= 1, n++) {
          bits--;
          if (put_bit(w, pos, (unsigned)(x & 1u))) break;
        }
      } else {
        break;
      }
    }
  }
  return maxbits - bits;
}

unsigned orc_encode_iblock(uint64_t* w, uint64_t* pos, unsigned minbits, unsigned maxbits, unsigned maxprec,
                           int32_t* q, unsigned dims)
{
  /* encode.c:412-455 */
  unsigned size = 1u << (2 * dims);
  uint32_t u[256];
  orc_fwd_xform(q, dims);
  orc_fwd_reorder(u, q, dims);
  unsigned budget = exceeded_maxbits(maxbits, maxprec, size) ? maxbits : ~0u;
  unsigned bits = orc_encode_ints(w, pos, u, budget, maxprec, size);
  if (bits < minbits) {
    *pos += minbits - bits; /* stream_pad: zero bits */
    bits = minbits;
  }
  return bits;
}

unsigned orc_encode_fblock(uint64_t* w, uint64_t* pos, const orc_params* p, const float* f, unsigned dims)
{
  /* encode.c:457-495 */
  unsigned bits = 1;
  unsigned size = 1u << (2 * dims);
  int emax = orc_block_exponent(f, size);
  unsigned maxprec = orc_precision(emax, p->maxprec, p->minexp, dims);
  unsigned e = maxprec ? (unsigned)(emax + EBIAS) : 0;
  if (e) {
    int32_t q[256];
    bits += EBITS;
    put_bits(w, pos, 2 * (uint64_t)e + 1, bits);
    orc_fwd_cast(q, f, size, emax);
    bits += orc_encode_iblock(w, pos, p->minbits - OMIN(bits, p->minbits), p->maxbits - bits, maxprec, q, dims);
  } else {
    put_bit(w, pos, 0);
    if (p->minbits > bits) {
      *pos += p->minbits - bits;
      bits = p->minbits;
    }
  }
  return bits;
}

/* ------------------------------------------------------------------------------------------------
 * Gather / scatter with partial-block padding (encode.c:41-126, decode.c:27-42)
 * ---------------------------------------------------------------------------------------------- */
static inline size_t pad_index(size_t i, size_t nvalid)
{
  /* pad_partial_block fall-through (encode.c:41-60): n=1 -> v0 v0 v0 v0; n=2 -> v0 v1 v1 v0; n=3 -> v0 v1 v2 v0 */
  switch (nvalid) {
    case 1: return 0;
    case 2: return i == 3 ? 0 : (i == 2 ? 1 : i);
    case 3: return i == 3 ? 0 : i;
    default: return i;
  }
}

static inline float load_value(const void* data, int dtype, ptrdiff_t off)
{
  if (dtype == ORC_BF16) {
    uint32_t b = (uint32_t)((const uint16_t*)data)[off] << 16;
    float f;
    memcpy(&f, &b, 4);
    return f;
  }
  return ((const float*)data)[off];
}

static void default_strides(unsigned dims, const size_t* n, const ptrdiff_t* s, ptrdiff_t* out)
{
  out[0] = s && s[0] ? s[0] : 1;
  out[1] = s && dims > 1 && s[1] ? s[1] : (ptrdiff_t)n[0];
  out[2] = s && dims > 2 && s[2] ? s[2] : (ptrdiff_t)(n[0] * (dims > 1 ? n[1] : 1));
  out[3] = s && dims > 3 && s[3] ? s[3] : (ptrdiff_t)(n[0] * (dims > 1 ? n[1] : 1) * (dims > 2 ? n[2] : 1));
}

void orc_gather_block(float* block, const void* data, int dtype, unsigned dims, const size_t* n,
                      const ptrdiff_t* s, const size_t* b)
{
  /* gather_partial_4d_block (encode.c:90-126) generalised: pad each axis in turn */
  ptrdiff_t st[4];
  default_strides(dims, n, s, st);
  size_t nv[4] = {1, 1, 1, 1};
  for (unsigned a = 0; a < dims; a++) nv[a] = OMIN((size_t)4, n[a] - 4 * b[a]);
  unsigned ew = dims > 3 ? 4 : 1, ez = dims > 2 ? 4 : 1, ey = dims > 1 ? 4 : 1;
  for (unsigned t = 0; t < ew; t++)
    for (unsigned z = 0; z < ez; z++)
      for (unsigned y = 0; y < ey; y++)
        for (unsigned x = 0; x < 4; x++) {
          ptrdiff_t off = (ptrdiff_t)(4 * b[0] + pad_index(x, nv[0])) * st[0];
          if (dims > 1) off += (ptrdiff_t)(4 * b[1] + pad_index(y, nv[1])) * st[1];
          if (dims > 2) off += (ptrdiff_t)(4 * b[2] + pad_index(z, nv[2])) * st[2];
          if (dims > 3) off += (ptrdiff_t)(4 * b[3] + pad_index(t, nv[3])) * st[3];
          block[64 * t + 16 * z + 4 * y + x] = load_value(data, dtype, off);
        }
}

static void scatter_block(const float* block, float* data, unsigned dims, const size_t* n, const ptrdiff_t* st,
                          const size_t* b)
{
  size_t nv[4] = {1, 1, 1, 1};
  for (unsigned a = 0; a < dims; a++) nv[a] = OMIN((size_t)4, n[a] - 4 * b[a]);
  for (unsigned t = 0; t < nv[3]; t++)
    for (unsigned z = 0; z < nv[2]; z++)
      for (unsigned y = 0; y < nv[1]; y++)
        for (unsigned x = 0; x < nv[0]; x++) {
          ptrdiff_t off = (ptrdiff_t)(4 * b[0] + x) * st[0];
          if (dims > 1) off += (ptrdiff_t)(4 * b[1] + y) * st[1];
          if (dims > 2) off += (ptrdiff_t)(4 * b[2] + z) * st[2];
          if (dims > 3) off += (ptrdiff_t)(4 * b[3] + t) * st[3];
          data[off] = block[64 * t + 16 * z + 4 * y + x];
        }
}

/* ------------------------------------------------------------------------------------------------
 * Array driver (zfp.c:10-56): traversal z, y, x; flush to 64 bits.
 * ---------------------------------------------------------------------------------------------- */
size_t orc_num_blocks(unsigned dims, const size_t* n)
{
  size_t nb = 1;
  for (unsigned a = 0; a < dims; a++) nb *= (n[a] + 3) / 4;
  return nb;
}

static inline void block_coords(size_t idx, unsigned dims, const size_t* n, size_t* b)
{
  size_t bx = (n[0] + 3) / 4;
  size_t by = dims > 1 ? (n[1] + 3) / 4 : 1;
  size_t bz = dims > 2 ? (n[2] + 3) / 4 : 1;
  b[0] = idx % bx;
  b[1] = (idx / bx) % by;
  b[2] = (idx / (bx * by)) % bz;
  b[3] = idx / (bx * by * bz);
}

static uint64_t compress_range(const void* data, int dtype, unsigned dims, const size_t* n, const ptrdiff_t* s,
                               const orc_params* p, size_t first, size_t last, uint64_t* out)
{
  uint64_t pos = 0;
  float f[256];
  size_t b[4];
  for (size_t i = first; i < last; i++) {
    block_coords(i, dims, n, b);
    orc_gather_block(f, data, dtype, dims, n, s, b);
    orc_encode_fblock(out, &pos, p, f, dims);
  }
  return pos;
}

static size_t max_block_bits(const orc_params* p, unsigned dims)
{
  unsigned size = 1u << (2 * dims);
  size_t mb = 9 + (size - 1) + (size_t)size * OMIN(p->maxprec, 32u); /* common.c:187-224 */
  if (p->maxbits >= 9) mb = OMIN(mb, (size_t)p->maxbits);
  return OMAX(mb, (size_t)p->minbits);
}

uint64_t orc_compress(const void* data, int dtype, unsigned dims, const size_t* n, const ptrdiff_t* s,
                      const orc_params* p, uint64_t* out, size_t out_words)
{
  memset(out, 0, out_words * 8);
  return compress_range(data, dtype, dims, n, s, p, 0, orc_num_blocks(dims, n), out);
}

typedef struct {
  const void* data;
  int dtype;
  unsigned dims;
  const size_t* n;
  const ptrdiff_t* s;
  const orc_params* p;
  size_t first, last;
  uint64_t* buf;
  uint64_t bits;
} shard_job;

static void* shard_main(void* arg)
{
  shard_job* j = (shard_job*)arg;
  j->bits = compress_range(j->data, j->dtype, j->dims, j->n, j->s, j->p, j->first, j->last, j->buf);
  return NULL;
}

static void stitch(uint64_t* out, uint64_t off, const uint64_t* src, uint64_t bits)
{
  /* Append `bits` bits of src at bit offset `off` (out zeroed). */
  uint64_t nw = (bits + 63) / 64;
  unsigned sh = (unsigned)(off & 63);
  uint64_t base = off >> 6;
  for (uint64_t i = 0; i < nw; i++) {
    uint64_t v = src[i];
    if (i == nw - 1 && (bits & 63)) v &= ((uint64_t)1 << (bits & 63)) - 1;
    out[base + i] |= v << sh;
    if (sh) {
      uint64_t hi = v >> (64 - sh);
      if (hi) out[base + i + 1] |= hi;
    }
  }
}

void orc_stitch(uint64_t* out, uint64_t off, const uint64_t* src, uint64_t bits) { stitch(out, off, src, bits); }

static int clamp_threads(int nthreads, size_t nb)
{
  if (nthreads < 1) nthreads = 1;
  if ((size_t)nthreads > nb) nthreads = (int)(nb ? nb : 1);
  return nthreads;
}

uint64_t orc_compress_mt(const void* data, int dtype, unsigned dims, const size_t* n, const ptrdiff_t* s,
                         const orc_params* p, uint64_t* out, size_t out_words, int nthreads)
{
  return orc_compress_mt_off(data, dtype, dims, n, s, p, out, out_words, nthreads, NULL);
}

/* Threaded encode: shard t = blocks [t * per, (t + 1) * per), per = ceil(nb / T), encoded independently and
 * stitched in order. shard_off (optional, T + 1 entries, T = the clamped thread count) receives each shard's first
 * bit in the stitched stream -- the split points orc_decompress_mt resumes at. */
uint64_t orc_compress_mt_off(const void* data, int dtype, unsigned dims, const size_t* n, const ptrdiff_t* s,
                             const orc_params* p, uint64_t* out, size_t out_words, int nthreads, uint64_t* shard_off)
{
  size_t nb = orc_num_blocks(dims, n);
  nthreads = clamp_threads(nthreads, nb);
  shard_job* jobs = (shard_job*)calloc((size_t)nthreads, sizeof(shard_job));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  size_t per = (nb + nthreads - 1) / nthreads;
  size_t mbb = max_block_bits(p, dims);
  for (int t = 0; t < nthreads; t++) {
    shard_job* j = &jobs[t];
    j->data = data; j->dtype = dtype; j->dims = dims; j->n = n; j->s = s; j->p = p;
    j->first = OMIN(nb, (size_t)t * per);
    j->last = OMIN(nb, j->first + per);
    size_t words = ((j->last - j->first) * mbb + 63) / 64 + 2;
    j->buf = (uint64_t*)calloc(words, 8);
    pthread_create(&th[t], NULL, shard_main, j);
  }
  memset(out, 0, out_words * 8);
  uint64_t off = 0;
  for (int t = 0; t < nthreads; t++) {
    pthread_join(th[t], NULL);
    if (shard_off) shard_off[t] = off;
    stitch(out, off, jobs[t].buf, jobs[t].bits);
    off += jobs[t].bits;
    free(jobs[t].buf);
  }
  if (shard_off) shard_off[nthreads] = off;
  free(jobs);
  free(th);
  return off;
}

void orc_block_bits(const void* data, int dtype, unsigned dims, const size_t* n, const ptrdiff_t* s,
                    const orc_params* p, uint32_t* bits_out)
{
  size_t nb = orc_num_blocks(dims, n);
  uint64_t scratch[300];
  float f[256];
  size_t b[4];
  for (size_t i = 0; i < nb; i++) {
    uint64_t pos = 0;
    memset(scratch, 0, sizeof(scratch));
    block_coords(i, dims, n, b);
    orc_gather_block(f, data, dtype, dims, n, s, b);
    bits_out[i] = orc_encode_fblock(scratch, &pos, p, f, dims);
  }
}

/* ------------------------------------------------------------------------------------------------
 * Decoder (libzfp 0.5.5 semantics; sw/src/decode.c:113-253 with block size 4^d)
 * ---------------------------------------------------------------------------------------------- */
/* decode.c:141-183 for 256 coefficients */
static unsigned decode_ints_256(const uint64_t* w, uint64_t* pos, unsigned maxbits, unsigned maxprec, uint32_t* u)
{
  unsigned intprec = 32;
  unsigned kmin = intprec > maxprec ? intprec - maxprec : 0;
  unsigned bits = maxbits;
  unsigned i, k, m, n;
  for (i = 0; i < 256; i++) u[i] = 0;
  for (k = intprec, n = 0; bits && k-- > kmin;) {
    m = OMIN(n, bits);
    bits -= m;
    uint64_t x[4] = {0, 0, 0, 0};
    for (unsigned o = 0; o < m; o += 64) x[o >> 6] = get_bits(w, pos, OMIN(64u, m - o));
    for (; n < 256 && bits && (bits--, get_bit(w, pos)); x[n >> 6] |= (uint64_t)1 << (n & 63), n++)
      for (; n < 255 && bits && (bits--, !get_bit(w, pos)); n++)
        ;
    for (i = 0; i < 256; i++) u[i] += (uint32_t)((x[i >> 6] >> (i & 63)) & 1u) << k;
  }
  return maxbits - bits;
}

static unsigned decode_ints(const uint64_t* w, uint64_t* pos, unsigned maxbits, unsigned maxprec, uint32_t* u,
                            unsigned size)
{
  if (size == 256) return decode_ints_256(w, pos, maxbits, maxprec, u);
  /* decode.c:141-183 */
  unsigned intprec = 32;
  unsigned kmin = intprec > maxprec ? intprec - maxprec : 0;
  unsigned bits = maxbits;
  unsigned i, k, m, n;
  for (i = 0; i < size; i++) u[i] = 0;
  for (k = intprec, n = 0; bits && k-- > kmin;) {
    m = OMIN(n, bits);
    bits -= m;
    uint64_t x = get_bits(w, pos, m);
    for (; n < size && bits && (bits--, get_bit(w, pos)); x += (uint64_t)1 << n++)
      for (; n < size - 1 && bits && (bits--, !get_bit(w, pos)); n++)
        ;
    for (i = 0; x; i++, x >>= 1) u[i] += (uint32_t)(x & 1u) << k;
  }
  return maxbits - bits;
}

static unsigned decode_fblock(const uint64_t* w, uint64_t* pos, const orc_params* p, float* f, unsigned dims)
{
  /* decode.c:220-253 + decode_iblock :185-218 */
  unsigned size = 1u << (2 * dims);
  unsigned bits = 1;
  if (get_bit(w, pos)) {
    bits += EBITS;
    int emax = (int)get_bits(w, pos, EBITS) - EBIAS;
    unsigned maxprec = orc_precision(emax, p->maxprec, p->minexp, dims);
    unsigned minb = p->minbits - OMIN(bits, p->minbits);
    unsigned maxb = p->maxbits - bits;
    uint32_t u[256];
    int32_t q[256];
    unsigned budget = exceeded_maxbits(maxb, maxprec, size) ? maxb : ~0u;
    unsigned got = decode_ints(w, pos, budget, maxprec, u, size);
    if (got < minb) {
      *pos += minb - got;
      got = minb;
    }
    bits += got;
    const unsigned char* perm = orc_perm(dims);
    for (unsigned i = 0; i < size; i++) q[perm[i]] = (int32_t)((u[i] ^ NBMASK) - NBMASK); /* decode.c:44-56 */
    orc_inv_xform(q, dims);
    float sc = ldexpf(1.0f, emax - 30); /* decode.c:12-25 dequantize */
    for (unsigned i = 0; i < size; i++) f[i] = (float)(sc * (float)q[i]);
  } else {
    for (unsigned i = 0; i < size; i++) f[i] = 0;
    if (p->minbits > bits) {
      *pos += p->minbits - bits;
      bits = p->minbits;
    }
  }
  return bits;
}

uint64_t orc_decompress(float* data, unsigned dims, const size_t* n, const ptrdiff_t* s, const orc_params* p,
                        const uint64_t* in, size_t in_words)
{
  (void)in_words;
  ptrdiff_t st[4];
  default_strides(dims, n, s, st);
  size_t nb = orc_num_blocks(dims, n);
  uint64_t pos = 0;
  float f[256];
  size_t b[4];
  for (size_t i = 0; i < nb; i++) {
    block_coords(i, dims, n, b);
    decode_fblock(in, &pos, p, f, dims);
    scatter_block(f, data, dims, n, st, b);
  }
  return pos;
}

static uint64_t decompress_range(float* data, unsigned dims, const size_t* n, const ptrdiff_t* st, const orc_params* p,
                                 const uint64_t* in, size_t first, size_t last, uint64_t pos)
{
  float f[256];
  size_t b[4];
  for (size_t i = first; i < last; i++) {
    block_coords(i, dims, n, b);
    decode_fblock(in, &pos, p, f, dims);
    scatter_block(f, data, dims, n, st, b);
  }
  return pos;
}

uint64_t orc_decompress_at(float* data, unsigned dims, const size_t* n, const ptrdiff_t* s, const orc_params* p,
                           const uint64_t* in, size_t in_words, uint64_t start_bit)
{
  (void)in_words;
  ptrdiff_t st[4];
  default_strides(dims, n, s, st);
  return decompress_range(data, dims, n, st, p, in, 0, orc_num_blocks(dims, n), start_bit);
}

typedef struct {
  float* data;
  unsigned dims;
  const size_t* n;
  const ptrdiff_t* st;
  const orc_params* p;
  const uint64_t* in;
  size_t first, last;
  uint64_t pos;
} dshard_job;

static void* dshard_main(void* arg)
{
  dshard_job* j = (dshard_job*)arg;
  j->pos = decompress_range(j->data, j->dims, j->n, j->st, j->p, j->in, j->first, j->last, j->pos);
  return NULL;
}

/* Threaded decode with the shard split of orc_compress_mt_off: shard t (blocks [t * per, (t + 1) * per)) starts at
 * bit shard_off[t]. shard_off may be NULL for fixed-rate streams (block i starts at i * maxbits). Every thread decodes
 * with the sequential decoder; returns the end bit of the last shard. */
uint64_t orc_decompress_mt(float* data, unsigned dims, const size_t* n, const ptrdiff_t* s, const orc_params* p,
                           const uint64_t* in, size_t in_words, int nthreads, const uint64_t* shard_off)
{
  (void)in_words;
  ptrdiff_t st[4];
  default_strides(dims, n, s, st);
  size_t nb = orc_num_blocks(dims, n);
  nthreads = clamp_threads(nthreads, nb);
  if (!shard_off && p->minbits != p->maxbits) nthreads = 1;
  size_t per = (nb + nthreads - 1) / nthreads;
  dshard_job* jobs = (dshard_job*)calloc((size_t)nthreads, sizeof(dshard_job));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) {
    dshard_job* j = &jobs[t];
    j->data = data; j->dims = dims; j->n = n; j->st = st; j->p = p; j->in = in;
    j->first = OMIN(nb, (size_t)t * per);
    j->last = OMIN(nb, j->first + per);
    j->pos = shard_off ? shard_off[t] : (uint64_t)j->first * p->maxbits;
    pthread_create(&th[t], NULL, dshard_main, j);
  }
  uint64_t end = 0;
  for (int t = 0; t < nthreads; t++) {
    pthread_join(th[t], NULL);
    end = jobs[t].pos;
  }
  free(jobs);
  free(th);
  return end;
}

/* ------------------------------------------------------------------------------------------------
 * zfp stream header (third-party format: LLNL zfp 0.5.5 src/zfp.c zfp_write_header / zfp_read_header,
 * zfp_field_metadata, zfp_stream_mode, zfp_stream_set_mode; the format zfpy.compress_numpy writes, which the
 * reference caller hw/models/train_imagenet.py:459-465 produces). Not implemented by sw/ (ZFP_HEADER_* in
 * sw/include/common.h:16-21 are declared and unused). Pinned by libzfp-generated fixtures
 * (tests/golden/libzfp_headers.json).
 * ---------------------------------------------------------------------------------------------- */
#define ORC_MIN_BITS 1u
#define ORC_MAX_BITS 16657u
#define ORC_MAX_PREC 64u
#define ORC_MIN_EXP (-1074)

static uint64_t field_meta(unsigned dims, const size_t* n, unsigned zfp_type)
{
  /* sizes (48 bits: 48 / 24 / 16 / 12 per axis by dims), then dims - 1 (2 bits), then type - 1 (2 bits) */
  uint64_t meta = 0;
  unsigned w = dims == 1 ? 48 : dims == 2 ? 24 : dims == 3 ? 16 : 12;
  for (int a = (int)dims - 1; a >= 0; a--) meta = (meta << w) + (uint64_t)(n[a] - 1);
  meta = (meta << 2) + (dims - 1);
  meta = (meta << 2) + (zfp_type - 1);
  return meta;
}

static uint64_t stream_mode(const orc_params* p)
{
  /* compression-mode classification (zfp_stream_compression_mode), then the short 12-bit forms for the three
   * standard modes, else four packed fields + 0xfff */
  const int valid = p->minbits <= p->maxbits && p->maxprec >= 1 && p->maxprec <= 64;
  const int dflt = p->minbits == ORC_MIN_BITS && p->maxbits == ORC_MAX_BITS && p->maxprec == ORC_MAX_PREC &&
                   p->minexp == ORC_MIN_EXP;
  if (valid && !dflt) {
    if (p->minbits == p->maxbits && p->maxbits >= 1 && p->maxbits <= ORC_MAX_BITS && p->maxprec >= ORC_MAX_PREC &&
        p->minexp <= ORC_MIN_EXP) {
      if (p->maxbits <= 2048) return (uint64_t)(p->maxbits - 1);
    } else if (p->minbits <= ORC_MIN_BITS && p->maxbits >= ORC_MAX_BITS && p->maxprec >= 1 &&
               p->minexp <= ORC_MIN_EXP) {
      if (p->maxprec <= 128) return (uint64_t)(p->maxprec - 1) + 2048;
    } else if (p->minbits <= ORC_MIN_BITS && p->maxbits >= ORC_MAX_BITS && p->maxprec >= ORC_MAX_PREC &&
               p->minexp >= ORC_MIN_EXP) {
      if (p->minexp <= 843) return (uint64_t)(p->minexp - ORC_MIN_EXP) + (2048 + 128 + 1);
    }
  }
  uint64_t minbits = OMAX(1u, OMIN(p->minbits, 0x8000u)) - 1;
  uint64_t maxbits = OMAX(1u, OMIN(p->maxbits, 0x8000u)) - 1;
  uint64_t maxprec = OMAX(1u, OMIN(p->maxprec, 0x0080u)) - 1;
  uint64_t minexp = (uint64_t)OMAX(0, OMIN(p->minexp + 16495, 0x7fff));
  uint64_t mode = minexp;
  mode = (mode << 7) + maxprec;
  mode = (mode << 15) + maxbits;
  mode = (mode << 15) + minbits;
  mode = (mode << 12) + 0xfffu;
  return mode;
}

unsigned orc_header_bits(const orc_params* p) { return stream_mode(p) < 0xfffu ? 96u : 148u; }

unsigned orc_write_header(uint64_t* words, unsigned dims, const size_t* n, unsigned zfp_type, const orc_params* p)
{
  uint64_t pos = 0;
  put_bits(words, &pos, 'z', 8);
  put_bits(words, &pos, 'f', 8);
  put_bits(words, &pos, 'p', 8);
  put_bits(words, &pos, 5, 8); /* zfp_codec_version of zfp 0.5.5 */
  put_bits(words, &pos, field_meta(dims, n, zfp_type), 52);
  uint64_t mode = stream_mode(p);
  put_bits(words, &pos, mode, mode < 0xfffu ? 12 : 64);
  return (unsigned)pos;
}

unsigned orc_read_header(const uint64_t* words, unsigned* dims, size_t* n, unsigned* zfp_type, orc_params* p)
{
  uint64_t pos = 0;
  if (get_bits(words, &pos, 8) != 'z' || get_bits(words, &pos, 8) != 'f' || get_bits(words, &pos, 8) != 'p' ||
      get_bits(words, &pos, 8) != 5)
    return 0;
  uint64_t meta = get_bits(words, &pos, 52);
  *zfp_type = (unsigned)(meta & 3u) + 1;
  meta >>= 2;
  *dims = (unsigned)(meta & 3u) + 1;
  meta >>= 2;
  unsigned w = *dims == 1 ? 48 : *dims == 2 ? 24 : *dims == 3 ? 16 : 12;
  for (unsigned a = 0; a < 4; a++) n[a] = 0;
  for (unsigned a = 0; a < *dims; a++) {
    n[a] = (size_t)(meta & ((1ull << w) - 1)) + 1;
    meta >>= w;
  }
  uint64_t mode = get_bits(words, &pos, 12);
  if (mode < 0xfffu) {
    if (mode < 2048) {
      p->minbits = p->maxbits = (unsigned)mode + 1;
      p->maxprec = ORC_MAX_PREC;
      p->minexp = ORC_MIN_EXP;
    } else if (mode < 2048 + 128) {
      p->minbits = ORC_MIN_BITS;
      p->maxbits = ORC_MAX_BITS;
      p->maxprec = (unsigned)mode + 1 - 2048;
      p->minexp = ORC_MIN_EXP;
    } else {
      p->minbits = ORC_MIN_BITS;
      p->maxbits = ORC_MAX_BITS;
      p->maxprec = ORC_MAX_PREC;
      p->minexp = (int)mode + ORC_MIN_EXP - (2048 + 128 + 1);
    }
  } else {
    mode += get_bits(words, &pos, 52) << 12;
    mode >>= 12;
    p->minbits = (unsigned)(mode & 0x7fffu) + 1;
    mode >>= 15;
    p->maxbits = (unsigned)(mode & 0x7fffu) + 1;
    mode >>= 15;
    p->maxprec = (unsigned)(mode & 0x7fu) + 1;
    mode >>= 7;
    p->minexp = (int)(mode & 0x7fffu) - 16495;
  }
  return (unsigned)pos;
}

/* ------------------------------------------------------------------------------------------------
 * Deterministic inputs
 * ---------------------------------------------------------------------------------------------- */
void orc_gen_bump2d(float* out, size_t n, int f32sum)
{
  /* sw/tests/test_zfp.cpp:13-25; f32sum: x*x + y*y summed in float32 (recipe that reproduces the
   * 530/550/590/600 goldens) */
  for (size_t j = 0; j < n; j++)
    for (size_t i = 0; i < n; i++) {
      double x = 2.0 * i / n;
      double y = 2.0 * j / n;
      if (f32sum) {
        float xf = (float)x, yf = (float)y;
        float r = xf * xf + yf * yf;
        out[i + n * j] = (float)exp(-(double)r);
      } else {
        out[i + n * j] = (float)exp(-(x * x + y * y));
      }
    }
}

static inline uint64_t splitmix64(uint64_t* st)
{
  uint64_t z = (*st += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void orc_gen_normal(float* out, size_t count, double sigma, uint64_t seed, int inject)
{
  /* splitmix64, Box-Muller in double then cast; injected zero / tiny (INT_MIN path) / subnormal
   * 4-value blocks at rates 1/64, 1/4096, 1/4096. */
  uint64_t st = seed;
  for (size_t i = 0; i < count; i += 2) {
    double u1 = ((double)(splitmix64(&st) >> 11) + 1.0) * 0x1.0p-53;
    double u2 = (double)(splitmix64(&st) >> 11) * 0x1.0p-53;
    double r = sqrt(-2.0 * log(u1));
    out[i] = (float)(sigma * r * cos(6.283185307179586 * u2));
    if (i + 1 < count) out[i + 1] = (float)(sigma * r * sin(6.283185307179586 * u2));
  }
  if (!inject) return;
  for (size_t blk = 0; blk * 4 < count; blk++) {
    uint64_t h = blk ^ seed;
    h = splitmix64(&h);
    double scale;
    if (h % 64 == 0) scale = 0.0;
    else if (h % 4096 == 1) scale = 1e-35 / sigma;
    else if (h % 4096 == 2) scale = 1e-40 / sigma;
    else continue;
    for (size_t k = 4 * blk; k < count && k < 4 * blk + 4; k++) out[k] = (float)((double)out[k] * scale);
  }
}
