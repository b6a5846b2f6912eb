// gcow_api.cpp -- libgcow.so: the C ABI declared in include/gcow.h.
//
// Part 1 keeps fpgasystems/gcow's sw/ call surface (sw/include/{types,zfp,stream,encode,decode}.h) with the same
// names, struct layouts, argument meaning and return values; the codec work behind it runs on the GPU through the
// device API of Part 2. There is no CPU codec here: host code only moves bytes (H<->D copies, stream bookkeeping,
// block gathers) and launches the gfx950 kernels in gcow_kernels.hip.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "gcow.h"
#include "kernels.h"

namespace {

thread_local std::string g_err;

gcow_status fail(gcow_status s, const std::string& msg)
{
  g_err = msg;
  return s;
}

gcow_status hipfail(hipError_t e, const char* where)
{
  g_err = std::string(where) + ": " + hipGetErrorString(e);
  return GCOW_ERR_HIP;
}

#define GCOW_HIP(call)                                  \
  do {                                                  \
    hipError_t e_ = (call);                             \
    if (e_ != hipSuccess) return hipfail(e_, #call);    \
  } while (0)

uint32_t dims_of(const zfp_input* in)
{
  // sw/src/common.c:122-125, extended with 1-D (nx set, ny == 0).
  return in->nx ? (in->ny ? (in->nz ? (in->nw ? 4u : 3u) : 2u) : 1u) : 0u;
}

bool is_device_ptr(const void* p)
{
  if (!p) return false;
  hipPointerAttribute_t a;
  hipError_t e = hipPointerGetAttributes(&a, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

// Tight per-block bit bound (sw/src/common.c:187-224 without the header term): max(minbits, min(maxbits,
// 9 + B - 1 + B * min(maxprec, 32))).
uint64_t block_bits_bound(const gcow_params& p, uint32_t dims)
{
  const uint64_t B = 1ull << (2 * dims);
  uint64_t mb = 9 + (B - 1) + B * std::min<uint64_t>(p.maxprec, 32);
  mb = std::min<uint64_t>(mb, p.maxbits);
  return std::max<uint64_t>(mb, std::max<uint64_t>(p.minbits, 1));
}

gcow_status make_field(const zfp_input* in, gcow::FieldDesc& F, bool for_decode, bool bf16_out = false)
{
  if (!in) return fail(GCOW_ERR_INVALID, "null field");
  const uint32_t d = dims_of(in);
  if (d == 0) return fail(GCOW_ERR_INVALID, "field has no extents");

  if (for_decode) {
    if (in->dtype != dtype_float && !(bf16_out && in->dtype == dtype_bf16))
      return fail(GCOW_ERR_UNSUPPORTED, bf16_out ? "decode writes dtype_float, or dtype_bf16 for 1-D fields"
                                                 : "decode writes fp32 (dtype_float) only");
  } else if (in->dtype != dtype_float && in->dtype != dtype_bf16) {
    return fail(GCOW_ERR_UNSUPPORTED, "encode supports dtype_float and dtype_bf16");
  }
  std::memset(&F, 0, sizeof(F));
  F.data = in->data;
  F.dims = d;
  F.dtype = in->dtype == dtype_bf16 ? gcow::DT_BF16 : gcow::DT_F32;
  F.n[0] = in->nx;
  F.n[1] = d > 1 ? in->ny : 1;
  F.n[2] = d > 2 ? in->nz : 1;
  F.n[3] = d > 3 ? in->nw : 1;
  F.s[0] = in->sx ? in->sx : 1;
  F.s[1] = d > 1 ? (in->sy ? in->sy : (ptrdiff_t)in->nx) : 0;
  F.s[2] = d > 2 ? (in->sz ? in->sz : (ptrdiff_t)(in->nx * in->ny)) : 0;
  F.s[3] = d > 3 ? (in->sw ? in->sw : (ptrdiff_t)(in->nx * in->ny * in->nz)) : 0;
  const uint64_t bx = (F.n[0] + 3) / 4, by = (F.n[1] + 3) / 4, bz = (F.n[2] + 3) / 4, bw = (F.n[3] + 3) / 4;
  const uint64_t nb = bx * by * bz * bw;
  if (nb >= (1ull << 32) || bx >= (1ull << 32)) return fail(GCOW_ERR_UNSUPPORTED, "more than 2^32 blocks per call");
  F.bx = (uint32_t)bx;
  F.by = (uint32_t)by;
  F.bz = (uint32_t)bz;
  F.bw = (uint32_t)bw;
  F.nblocks = (uint32_t)nb;
  const size_t esz = F.dtype == gcow::DT_BF16 ? 2 : 4;
  const bool aligned = ((uintptr_t)in->data % (4 * esz)) == 0;
  F.vec = (F.s[0] == 1 && aligned && (d < 2 || F.s[1] % 4 == 0) && (d < 3 || F.s[2] % 4 == 0) &&
           (d < 4 || F.s[3] % 4 == 0)) ? 1u : 0u;
  return GCOW_OK;
}

gcow_status check_params(const gcow_params* p, uint32_t dims)
{
  if (!p) return fail(GCOW_ERR_INVALID, "null params");
  if (p->maxbits < 9) return fail(GCOW_ERR_INVALID, "maxbits must be >= 9 (header + 1)");
  if (p->minbits > p->maxbits) return fail(GCOW_ERR_INVALID, "minbits > maxbits");
  if (block_bits_bound(*p, dims) > 20000) return fail(GCOW_ERR_UNSUPPORTED, "block bit bound above 20000");
  return GCOW_OK;
}

gcow::Params P(const gcow_params& p) { return gcow::Params{p.minbits, p.maxbits, p.maxprec, p.minexp}; }

gcow::TilePlan make_plan(const gcow::FieldDesc& F, const gcow_params& p)
{
  gcow::TilePlan pl;
  const uint64_t U = block_bits_bound(p, F.dims);
  pl.fixed = p.minbits == p.maxbits;
  pl.threads = F.dims == 3 ? 64 : (U <= 2048 ? 256 : 64);
  if (pl.fixed) {
    pl.range = pl.threads;
  } else if (F.dims == 3) {
    pl.range = 64;  // one 64-block tile per workgroup (gcow_blocks.hip k_count3d / k_encode3d_var)
  } else {
    const uint64_t target = 2048;
    uint64_t r = (F.nblocks + target - 1) / target;
    r = (r + pl.threads - 1) / pl.threads * pl.threads;
    pl.range = (uint32_t)std::max<uint64_t>(r, pl.threads);
  }
  pl.nranges = (uint32_t)((F.nblocks + pl.range - 1) / pl.range);
  pl.lds_words = (uint32_t)((31 + (uint64_t)pl.threads * U + 31) / 32 + 2);
  return pl;
}

bool fast1d_ok(const gcow::FieldDesc& F, const gcow_params& p, const uint64_t* d_index)
{
  return F.dims == 1 && F.vec && p.minbits == p.maxbits && (p.maxbits == 64 || p.maxbits == 32) && !d_index;
}

gcow_status encode_impl(const zfp_input* field, const gcow_params* p, void* d_out, size_t out_capacity,
                        uint64_t* d_total_bits, void* d_ws, size_t ws_bytes, uint64_t* d_index,
                        uint32_t index_stride, void* stream, const uint64_t* d_base = nullptr)
{
  gcow::FieldDesc F;
  gcow_status st = make_field(field, F, false);
  if (st) return st;
  if ((st = check_params(p, F.dims))) return st;
  if (!d_out) return fail(GCOW_ERR_INVALID, "null output");
  const size_t bound = gcow_max_output_bytes(field, p);
  if (out_capacity < bound) return fail(GCOW_ERR_CAPACITY, "output capacity below gcow_max_output_bytes()");
  uint32_t shift = 0;
  if (d_index) {
    if (!index_stride || index_stride > 256 || (index_stride & (index_stride - 1)))
      return fail(GCOW_ERR_INVALID, "index_stride must be a power of two in [1, 256]");
    while ((1u << shift) < index_stride) shift++;
  }
  if (d_base && p->minbits == p->maxbits)
    return fail(GCOW_ERR_UNSUPPORTED, "append with a device base offset is for variable-rate streams (fixed rate: "
                                      "offset the output pointer by nblocks * maxbits / 8 on the host)");
  if (F.nblocks == 0) {
    if (d_total_bits) {
      if (d_base) GCOW_HIP(hipMemcpyAsync(d_total_bits, d_base, 8, hipMemcpyDeviceToDevice, (hipStream_t)stream));
      else GCOW_HIP(gcow::launch_set_u64(d_total_bits, 0, stream));
    }
    return GCOW_OK;
  }
  const gcow::Params pp = P(*p);
  if (F.dims == 4) {  // one wave per 256-value block
    if (p->minbits == p->maxbits) {
      if (p->maxbits % 32) GCOW_HIP(hipMemsetAsync(d_out, 0, bound, (hipStream_t)stream));  // shared boundary words
      GCOW_HIP(gcow::launch_encode4d(F, pp, nullptr, nullptr, (uint32_t*)d_out, d_index, shift, stream));
      if (d_total_bits) GCOW_HIP(gcow::launch_set_u64(d_total_bits, (uint64_t)F.nblocks * p->maxbits, stream));
      return GCOW_OK;
    }
    const size_t need = gcow_encode_workspace_bytes(field, p);
    if (!d_ws || ws_bytes < need) return fail(GCOW_ERR_INVALID, "workspace smaller than gcow_encode_workspace_bytes()");
    uint64_t* sums = (uint64_t*)d_ws;
    uint64_t* base = sums + F.nblocks;
    uint32_t* lens = (uint32_t*)(base + F.nblocks + 1);
    GCOW_HIP(gcow::launch_encode4d(F, pp, lens, nullptr, nullptr, nullptr, 0, stream));
    GCOW_HIP(gcow::launch_scan_blocks(lens, F.nblocks, sums, base, d_total_bits, (uint32_t*)d_out, stream));
    GCOW_HIP(gcow::launch_encode4d(F, pp, nullptr, base, (uint32_t*)d_out, d_index, shift, stream));
    return GCOW_OK;
  }
  if (fast1d_ok(F, *p, d_index)) {
    GCOW_HIP(gcow::launch_encode_fixed1d(F.data, (int)F.dtype, F.n[0], F.nblocks, pp, d_out, stream));
    if (p->maxbits == 32 && (F.nblocks & 1))  // stream_flush: zero the upper half of the last word
      GCOW_HIP(hipMemsetAsync((uint32_t*)d_out + F.nblocks, 0, 4, (hipStream_t)stream));
    if (d_total_bits) GCOW_HIP(gcow::launch_set_u64(d_total_bits, (uint64_t)F.nblocks * p->maxbits, stream));
    return GCOW_OK;
  }
  if (F.dims == 3 && p->minbits == p->maxbits && !d_index && gcow::fixed3d_ok(p->maxbits)) {
    GCOW_HIP(gcow::launch_encode3d_fixed(F, pp, (uint32_t*)d_out, stream));
    if (d_total_bits) GCOW_HIP(gcow::launch_set_u64(d_total_bits, (uint64_t)F.nblocks * p->maxbits, stream));
    return GCOW_OK;
  }
  const gcow::TilePlan pl = make_plan(F, *p);
  uint64_t *sums = nullptr, *base = nullptr;
  if (!pl.fixed) {
    const size_t need = gcow_encode_workspace_bytes(field, p);
    if (!d_ws || ws_bytes < need) return fail(GCOW_ERR_INVALID, "workspace smaller than gcow_encode_workspace_bytes()");
    sums = (uint64_t*)d_ws;
    base = sums + pl.nranges;
  }
  GCOW_HIP(gcow::launch_encode_tiles(F, pp, pl, (uint32_t*)d_out, sums, base, pl.fixed ? nullptr : d_total_bits,
                                     d_index, shift, d_base, stream));
  if (pl.fixed && d_total_bits)
    GCOW_HIP(gcow::launch_set_u64(d_total_bits, (uint64_t)F.nblocks * p->maxbits, stream));
  return GCOW_OK;
}

gcow_status decode_impl(const zfp_input* field, const gcow_params* p, const void* d_in, const uint64_t* d_index,
                        uint32_t index_stride, uint64_t base_bits, uint64_t* d_end, void* stream,
                        size_t in_bytes = 0)
{
  gcow::FieldDesc F;
  gcow_status st = make_field(field, F, true, true);
  if (st) return st;
  if (F.dtype == gcow::DT_BF16 && F.dims != 1) return fail(GCOW_ERR_UNSUPPORTED, "bf16 output is for 1-D fields");
  if ((st = check_params(p, F.dims))) return st;
  if (!d_in) return fail(GCOW_ERR_INVALID, "null input stream");
  if (F.nblocks == 0) return GCOW_OK;
  const bool fixed = p->minbits == p->maxbits;
  if (fixed && F.dims == 1 && F.vec && (p->maxbits == 64 || p->maxbits == 32) && p->maxprec >= 32 &&
      p->minexp <= -154 && base_bits % 32 == 0 && !d_end) {
    GCOW_HIP(gcow::launch_decode_fixed1d(F, P(*p), (const uint64_t*)d_in, base_bits, stream));
    return GCOW_OK;
  }
  if (F.dims == 4) {  // one wave per block; a variable-rate stream without a stride-1 index is walked in order
    if ((!fixed && (!d_index || index_stride != 1)) || d_end)
      GCOW_HIP(gcow::launch_decode4d_seq(F, P(*p), (const uint64_t*)d_in, base_bits, d_end, stream));
    else
      GCOW_HIP(gcow::launch_decode4d(F, P(*p), (const uint64_t*)d_in, fixed ? nullptr : d_index, base_bits, stream));
    return GCOW_OK;
  }
  if (fixed && F.dims == 3 && base_bits % 32 == 0 && !d_end && gcow::fixed3d_ok(p->maxbits)) {
    GCOW_HIP(gcow::launch_decode3d_fixed(F, P(*p), (const uint32_t*)((const char*)d_in + base_bits / 8), stream));
    return GCOW_OK;
  }
  uint32_t chunk;
  uint64_t nchunks;
  if (fixed) {
    chunk = 1;
    nchunks = F.nblocks;
    d_index = nullptr;
  } else if (d_index) {
    if (!index_stride || (index_stride & (index_stride - 1)) || index_stride > 256)
      return fail(GCOW_ERR_INVALID, "index_stride must be a power of two in [1, 256]");
    chunk = index_stride;
    nchunks = (F.nblocks + chunk - 1) / chunk;
  } else {
    chunk = F.nblocks;  // no index: one sequential lane
    nchunks = 1;
  }
  if (!fixed && F.dims == 1 && F.vec && p->minbits <= 1 && p->maxbits >= 160) {
    GCOW_HIP(gcow::launch_decode1d_var(F, P(*p), (const uint64_t*)d_in, in_bytes / 8, d_index, chunk, nchunks,
                                       base_bits, d_end, stream));
    return GCOW_OK;
  }
  GCOW_HIP(gcow::launch_decode(F, P(*p), (const uint64_t*)d_in, d_index, chunk, nchunks, fixed, base_bits, d_end,
                               stream, in_bytes / 8));
  return GCOW_OK;
}

// ---------------------------------------------------------------------------------------------- drop-in state
// Device-side caches attached to a zfp_output (staging buffers, the device copy of its stream and the block index
// written by the last compress, so that a compress -> decompress round trip never re-uploads the stream).
struct OutState {
  void* d_stream = nullptr;
  size_t d_stream_cap = 0;
  void* d_data = nullptr;
  size_t d_data_cap = 0;
  uint64_t* d_index = nullptr;
  size_t d_index_cap = 0;
  void* d_ws = nullptr;
  size_t d_ws_cap = 0;
  uint64_t* d_u64 = nullptr;  // [0] total bits, [1] end position, [2] stream-compare flag
  // what the cached device stream holds
  bool valid = false;
  const void* host_begin = nullptr;
  uint64_t bits = 0;
  uint32_t index_stride = 0;
  gcow_params params{};
  uint32_t dims = 0;
  uint64_t nblocks = 0;
  uint64_t words = 0;
  std::vector<uint64_t> shadow;  // host streams: the caller's stream as zfp_compress left it (exact cache check)
};

std::mutex g_mu;
std::unordered_map<const zfp_output*, OutState*> g_states;

OutState* state_of(const zfp_output* o)
{
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_states.find(o);
  if (it != g_states.end()) return it->second;
  OutState* s = new OutState();
  g_states[o] = s;
  return s;
}

void drop_state(const zfp_output* o)
{
  OutState* s = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_states.find(o);
    if (it == g_states.end()) return;
    s = it->second;
    g_states.erase(it);
  }
  (void)hipFree(s->d_stream);
  (void)hipFree(s->d_data);
  (void)hipFree(s->d_index);
  (void)hipFree(s->d_ws);
  (void)hipFree(s->d_u64);
  delete s;
}

hipError_t grow(void** p, size_t* cap, size_t need)
{
  if (*cap >= need && *p) return hipSuccess;
  (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  hipError_t e = hipMalloc(p, need ? need : 8);
  if (e == hipSuccess) *cap = need;
  return e;
}

gcow_params params_of(const zfp_output* o) { return gcow_params{o->minbits, o->maxbits, o->maxprec, o->minexp}; }

// Element offsets [lo, hi] that a (possibly strided, possibly negatively strided) field touches, relative to its
// data pointer, with sw/'s stride defaults (sw/src/zfp.c:37-38: sx = 1, sy = nx, ...).
void field_span(const zfp_input* in, ptrdiff_t* lo, ptrdiff_t* hi)
{
  const uint32_t d = dims_of(in);
  const size_t n[4] = {in->nx, d > 1 ? in->ny : 1, d > 2 ? in->nz : 1, d > 3 ? in->nw : 1};
  const ptrdiff_t s[4] = {in->sx ? in->sx : 1, d > 1 ? (in->sy ? in->sy : (ptrdiff_t)in->nx) : 0,
                          d > 2 ? (in->sz ? in->sz : (ptrdiff_t)(in->nx * in->ny)) : 0,
                          d > 3 ? (in->sw ? in->sw : (ptrdiff_t)(in->nx * in->ny * in->nz)) : 0};
  *lo = *hi = 0;
  for (int k = 0; k < 4; k++) {
    const ptrdiff_t e = (ptrdiff_t)(n[k] ? n[k] - 1 : 0) * s[k];
    if (e < 0) *lo += e;
    else *hi += e;
  }
}

bool strided(const zfp_input* in) { return in->sx || in->sy || in->sz || in->sw; }

// Whole-stream check that the caller's buffer still holds the stream zfp_compress left in it (zfp_decompress reuses
// the device copy only then; a caller that rewrote its buffer -- another stream of the same shape, a local edit -- is
// decoded from its new contents). Host streams: a memcmp against a host shadow copy taken at compress time (exact, no
// hash collisions, and faster than hashing: one memcpy at compress, one memcmp at decompress). Device streams: every
// word compared on the device against the cached copy.

// Host-side copy of `bits` bits from words src into stream s at its current write position (stream.c:61-92).
void append_bits(stream* s, const uint64_t* src, uint64_t bits)
{
  uint64_t full = bits / 64;
  for (uint64_t i = 0; i < full; i++) stream_write_bits(s, src[i], 64);
  if (bits % 64) stream_write_bits(s, src[full] & ((1ull << (bits % 64)) - 1), bits % 64);
}

// Per-thread scratch for the block-API wrappers (small, synchronous calls).
struct Scratch {
  void* d = nullptr;
  size_t cap = 0;
  ~Scratch() { (void)hipFree(d); }
};
thread_local Scratch g_scratch;

void* scratch(size_t bytes)
{
  if (grow(&g_scratch.d, &g_scratch.cap, bytes) != hipSuccess) return nullptr;
  return g_scratch.d;
}

}  // namespace

extern "C" {

// ================================================================================================ misc
const uchar PERM_2D[16] = {0, 1, 4, 5, 2, 8, 6, 9, 3, 12, 10, 7, 13, 11, 14, 15};

const char* gcow_status_string(gcow_status s)
{
  switch (s) {
    case GCOW_OK: return "ok";
    case GCOW_ERR_INVALID: return "invalid argument";
    case GCOW_ERR_CAPACITY: return "output capacity too small";
    case GCOW_ERR_HIP: return "HIP runtime error";
    case GCOW_ERR_NODEVICE: return "no usable gfx950 device";
    case GCOW_ERR_UNSUPPORTED: return "unsupported";
  }
  return "unknown";
}

const char* gcow_last_error(void) { return g_err.c_str(); }
const char* gcow_version(void) { return "gcow-mi355x 0.1 (gfx950)"; }

// ================================================================================================ parameters
double set_zfp_output_accuracy(zfp_output* output, double tolerance)
{
  // sw/src/common.c:6-21
  int emin = ZFP_MIN_EXP;
  if (tolerance > 0) {
    (void)frexp(tolerance, &emin);
    emin--;
  }
  output->minbits = ZFP_MIN_BITS;
  output->maxbits = ZFP_MAX_BITS;
  output->maxprec = ZFP_MAX_PREC;
  output->minexp = emin;
  return tolerance > 0 ? ldexp(1.0, emin) : 0;
}

double set_zfp_output_rate(zfp_output* output, double rate, uint dim)
{
  // libzfp 0.5.5 zfp_stream_set_rate (no write-random-access), float: at least 1 + 8 bits per block
  uint n = 1u << (2 * dim);
  uint bits = (uint)floor(n * rate + 0.5);
  if (bits < 9) bits = 9;
  output->minbits = bits;
  output->maxbits = bits;
  output->maxprec = ZFP_MAX_PREC;
  output->minexp = ZFP_MIN_EXP;
  return (double)bits / n;
}

uint set_zfp_output_precision(zfp_output* output, uint precision)
{
  // libzfp 0.5.5 zfp_stream_set_precision
  output->minbits = ZFP_MIN_BITS;
  output->maxbits = ZFP_MAX_BITS;
  output->maxprec = precision ? (precision < ZFP_MAX_PREC ? precision : ZFP_MAX_PREC) : ZFP_MAX_PREC;
  output->minexp = ZFP_MIN_EXP;
  return output->maxprec;
}

int set_zfp_output_expert(zfp_output* output, uint minbits, uint maxbits, uint maxprec, int minexp)
{
  // libzfp 0.5.5 zfp_stream_set_params (returns 0 and leaves the stream intact on invalid input)
  if (minbits > maxbits || maxbits < 9 || !maxprec || maxprec > ZFP_MAX_PREC || minexp < ZFP_MIN_EXP) return 0;
  output->minbits = minbits;
  output->maxbits = maxbits;
  output->maxprec = maxprec;
  output->minexp = minexp;
  return 1;
}

zfp_input* alloc_zfp_input(void)
{
  zfp_input* in = (zfp_input*)malloc(sizeof(zfp_input));
  if (in) {
    in->dtype = dtype_none;
    in->nx = in->ny = in->nz = in->nw = 0;
    in->sx = in->sy = in->sz = in->sw = 0;
    in->data = NULL;
  }
  return in;
}

zfp_output* alloc_zfp_output(void)
{
  zfp_output* o = (zfp_output*)malloc(sizeof(zfp_output));
  if (o) {
    o->data = NULL;
    o->minbits = ZFP_MIN_BITS;
    o->maxbits = ZFP_MAX_BITS;
    o->maxprec = ZFP_MAX_PREC;
    o->minexp = ZFP_MIN_EXP;
  }
  return o;
}

void free_zfp_input(zfp_input* input)
{
  // sw/src/common.c:54-62 frees the caller's data; kept for host data, never for device memory.
  if (!input) return;
  if (input->data && !is_device_ptr(input->data)) free(input->data);
  free(input);
}

void free_zfp_output(zfp_output* output)
{
  if (!output) return;
  drop_state(output);
  if (output->data) {
    if (output->data->begin && !is_device_ptr(output->data->begin)) free(output->data->begin);
    free(output->data);
  }
  free(output);
}

void cleanup(zfp_input* input, zfp_output* output)
{
  free_zfp_input(input);
  free_zfp_output(output);
}

zfp_input* init_zfp_input(void* data, data_type dtype, uint dim, ...)
{
  // sw/src/common.c:83-103; dim 1 reads only nx.
  va_list shapes;
  va_start(shapes, dim);
  zfp_input* in = alloc_zfp_input();
  if (in) {
    in->data = data;
    in->dtype = dtype;
    in->nx = va_arg(shapes, uint);
    if (dim > 1) {
      in->ny = va_arg(shapes, uint);
      if (dim > 2) {
        in->nz = va_arg(shapes, uint);
        if (dim > 3) in->nw = va_arg(shapes, uint);
      }
    }
  }
  va_end(shapes);
  return in;
}

zfp_output* init_zfp_output(const zfp_input* input)
{
  // sw/src/common.c:105-115 (without the printf)
  zfp_output* o = alloc_zfp_output();
  if (!o) return NULL;
  size_t bytes = get_max_output_bytes(o, input);
  void* buf = malloc(bytes ? bytes : 8);
  o->data = stream_init(buf, bytes);
  if (o->data) stream_rewind(o->data);
  return o;
}

uint is_reversible(const zfp_output* output) { return output->minexp < ZFP_MIN_EXP; }

uint get_input_dimension(const zfp_input* input) { return dims_of(input); }

size_t get_input_num_blocks(const zfp_input* input)
{
  size_t bx = (input->nx + 3) / 4, by = (input->ny + 3) / 4, bz = (input->nz + 3) / 4, bw = (input->nw + 3) / 4;
  switch (dims_of(input)) {
    case 1: return bx;
    case 2: return bx * by;
    case 3: return bx * by * bz;
    case 4: return bx * by * bz * bw;
    default: return 0;
  }
}

size_t get_input_size(const zfp_input* input, size_t* shape)
{
  if (shape) switch (dims_of(input)) {
      case 4: shape[3] = input->nw; /* FALLTHROUGH */
      case 3: shape[2] = input->nz; /* FALLTHROUGH */
      case 2: shape[1] = input->ny; /* FALLTHROUGH */
      case 1: shape[0] = input->nx; break;
    }
  auto mx = [](size_t v) { return v ? v : (size_t)1; };
  return mx(input->nx) * mx(input->ny) * mx(input->nz) * mx(input->nw);
}

size_t get_dtype_size(data_type dtype)
{
  switch (dtype) {
    case dtype_int32: return 4;
    case dtype_int64: return 8;
    case dtype_float: return 4;
    case dtype_double: return 8;
    case dtype_bf16: return 2;
    default: return 0;
  }
}

uint get_input_precision(const zfp_input* input) { return (uint)(8 * get_dtype_size(input->dtype)); }

size_t get_max_output_bytes(const zfp_output* output, const zfp_input* input)
{
  // sw/src/common.c:187-224 (bf16 is coded as fp32)
  int reversible = is_reversible(output);
  uint dim = dims_of(input);
  size_t num_blocks = get_input_num_blocks(input);
  uint values = 1u << (2 * dim);
  uint maxbits = 0;
  if (!dim) return 0;
  uint prec = (uint)(8 * get_dtype_size(input->dtype));
  switch (input->dtype) {
    case dtype_int32: maxbits += reversible ? 5 : 0; break;
    case dtype_int64: maxbits += reversible ? 6 : 0; break;
    case dtype_float: maxbits += reversible ? 1 + 1 + 8 + 5 : 1 + 8; break;
    case dtype_bf16: maxbits += reversible ? 1 + 1 + 8 + 5 : 1 + 8; prec = 32; break;
    case dtype_double: maxbits += reversible ? 1 + 1 + 11 + 6 : 1 + 11; break;
    default: return 0;
  }
  maxbits += values - 1 + values * (output->maxprec < prec ? output->maxprec : prec);
  maxbits = maxbits < output->maxbits ? maxbits : output->maxbits;
  maxbits = maxbits > output->minbits ? maxbits : output->minbits;
  return ((ZFP_HEADER_MAX_BITS + num_blocks * maxbits + 63) & ~(size_t)63) / 8;
}

uint get_precision(int maxexp, uint maxprec, int minexp, int dim)
{
  int p = maxexp - minexp + 2 * dim + 2;
  uint up = p > 0 ? (uint)p : 0u;
  return maxprec < up ? maxprec : up;
}

int exceeded_maxbits(uint maxbits, uint maxprec, uint size) { return (maxprec + 1) * size - 1 > maxbits; }

// ================================================================================================ bit stream
// sw/src/stream.c semantics (host-side stream bookkeeping for the drop-in API).
static inline void sw_write_word(stream* s, stream_word v) { s->begin[s->idx++] = v; }
static inline stream_word sw_read_word(stream* s) { return s->begin[s->idx++]; }

stream* stream_init(void* buffer, size_t bytes)
{
  stream* s = (stream*)malloc(sizeof(stream));
  if (s) {
    s->begin = (stream_word*)buffer;
    s->end = (ptrdiff_t)(bytes / sizeof(stream_word));
    stream_rewind(s);
  }
  return s;
}

void stream_rewind(stream* s)
{
  s->idx = 0;
  s->buffer = 0;
  s->buffered_bits = 0;
}

size_t stream_size_bytes(const stream* s) { return (size_t)s->idx * sizeof(stream_word); }

stream_word stream_read_word(stream* s) { return sw_read_word(s); }
void stream_write_word(stream* s, stream_word value) { sw_write_word(s, value); }

uint64 stream_read_bits(stream* s, size_t n)
{
  uint64 value = s->buffer;
  if (s->buffered_bits < n) {
    s->buffer = sw_read_word(s);
    value += s->buffered_bits < 64 ? (uint64)s->buffer << s->buffered_bits : 0;
    s->buffered_bits += 64;
    s->buffered_bits -= n;
    if (!s->buffered_bits) {
      s->buffer = 0;
    } else {
      s->buffer >>= 64 - s->buffered_bits;
      value &= ((uint64)2 << (n - 1)) - 1;
    }
  } else {
    s->buffered_bits -= n;
    s->buffer = n < 64 ? s->buffer >> n : 0;
    value &= n < 64 ? ((uint64)1 << n) - 1 : ~(uint64)0;
  }
  return value;
}

uint64 stream_write_bits(stream* s, uint64 value, size_t n)
{
  if (n == 0) return value;
  s->buffer += (stream_word)(value << s->buffered_bits);
  s->buffered_bits += n;
  if (s->buffered_bits >= 64) {
    s->buffered_bits -= 64;
    sw_write_word(s, s->buffer);
    size_t sh = n - s->buffered_bits;
    s->buffer = sh < 64 ? (stream_word)(value >> sh) : 0;
  }
  s->buffer &= s->buffered_bits ? ((stream_word)1 << s->buffered_bits) - 1 : 0;
  return n < 64 ? value >> n : 0;
}

uint stream_read_bit(stream* s)
{
  if (!s->buffered_bits) {
    s->buffer = sw_read_word(s);
    s->buffered_bits = 64;
  }
  s->buffered_bits--;
  uint bit = (uint)s->buffer & 1u;
  s->buffer >>= 1;
  return bit;
}

uint stream_write_bit(stream* s, uint bit)
{
  s->buffer += (stream_word)bit << s->buffered_bits;
  if (++s->buffered_bits == 64) {
    sw_write_word(s, s->buffer);
    s->buffer = 0;
    s->buffered_bits = 0;
  }
  return bit;
}

void stream_pad(stream* s, uint64 n)
{
  uint64 bits = s->buffered_bits;
  for (bits += n; bits >= 64; bits -= 64) {
    sw_write_word(s, s->buffer);
    s->buffer = 0;
  }
  s->buffered_bits = (size_t)bits;
}

size_t stream_flush(stream* s)
{
  size_t bits = (64 - s->buffered_bits) % 64;
  if (bits) stream_pad(s, bits);
  return bits;
}

uint64 stream_woffset(stream* s) { return (uint64)s->idx * 64 + s->buffered_bits; }
uint64 stream_roffset(stream* s) { return (uint64)s->idx * 64 - s->buffered_bits; }

void stream_rseek(stream* s, uint64 offset)
{
  size_t n = (size_t)(offset % 64);
  s->idx = (ptrdiff_t)(offset / 64);
  if (n) {
    s->buffer = sw_read_word(s) >> n;
    s->buffered_bits = 64 - n;
  } else {
    s->buffer = 0;
    s->buffered_bits = 0;
  }
}

void stream_skip(stream* s, uint64 n) { stream_rseek(s, stream_roffset(s) + n); }

size_t stream_algin_next_word(stream* s)
{
  size_t bits = s->buffered_bits;
  if (bits) stream_skip(s, bits);
  return bits;
}

// ================================================================================================ device API
size_t gcow_max_output_bytes(const zfp_input* field, const gcow_params* p)
{
  const uint32_t d = dims_of(field);
  if (!d || d > 4 || !p) return 0;
  const uint64_t nb = get_input_num_blocks(field);
  return (size_t)((nb * block_bits_bound(*p, d) + 63) / 64 * 8 + 8);
}

size_t gcow_encode_workspace_bytes(const zfp_input* field, const gcow_params* p)
{
  gcow::FieldDesc F;
  if (make_field(field, F, false) || !p || p->minbits == p->maxbits) return 0;
  if (F.dims == 4) return (size_t)F.nblocks * 4 + (2 * (size_t)F.nblocks + 1) * 8 + 16;  // lens, sums, base
  const gcow::TilePlan pl = make_plan(F, *p);
  // sums, base; 3-D variable rate also keeps every block's length (uint16) from the count pass for the encode pass
  const size_t lens = F.dims == 3 ? ((size_t)F.nblocks * 2 + 7) / 8 * 8 : 0;
  const size_t two_pass = (2 * (size_t)pl.nranges + 1) * 8 + lens;
  // 1-D variable rate without a budget: the tile form's tile sums, offsets and byte lengths (the default), or the
  // single-pass encoder's look-back status and boundary words
  if (F.dims == 1 && pl.threads == 256 && p->minbits <= 1 && p->maxbits >= 160)
    return std::max({two_pass, gcow::var1d_sp_workspace_bytes(F.nblocks), gcow::var1d_tile_workspace_bytes(F.nblocks)});
  return two_pass;
}

size_t gcow_index_entries(const zfp_input* field, uint32_t index_stride)
{
  if (!index_stride) return 0;
  const uint64_t nb = get_input_num_blocks(field);
  return (size_t)((nb + index_stride - 1) / index_stride);
}

gcow_status gcow_encode_device(const zfp_input* field, const gcow_params* p, void* d_out, size_t out_capacity,
                               uint64_t* d_total_bits, void* d_workspace, size_t workspace_bytes, uint64_t* d_index,
                               uint32_t index_stride, void* hip_stream)
{
  return encode_impl(field, p, d_out, out_capacity, d_total_bits, d_workspace, workspace_bytes, d_index, index_stride,
                     hip_stream);
}

gcow_status gcow_encode_device_append(const zfp_input* field, const gcow_params* p, void* d_out, size_t out_capacity,
                                      const uint64_t* d_base_bits, uint64_t* d_total_bits, void* d_workspace,
                                      size_t workspace_bytes, uint64_t* d_index, uint32_t index_stride,
                                      void* hip_stream)
{
  if (!d_base_bits) return fail(GCOW_ERR_INVALID, "null base bit offset");
  return encode_impl(field, p, d_out, out_capacity, d_total_bits, d_workspace, workspace_bytes, d_index, index_stride,
                     hip_stream, d_base_bits);
}

gcow_status gcow_decode_device(const zfp_input* field, const gcow_params* p, const void* d_in, size_t in_bytes,
                               const uint64_t* d_index, uint32_t index_stride, void* hip_stream)
{
  return decode_impl(field, p, d_in, d_index, index_stride, 0, nullptr, hip_stream, in_bytes);
}

// ---------------------------------------------------------------------------------------------- zfp header
// Restates libzfp 0.5.5 zfp_field_metadata / zfp_stream_mode / zfp_write_header / zfp_read_header / zfp_stream_set_mode
// (third-party format; pinned by tests/golden/libzfp_headers.json).
static const uint32_t kMinBits = 1, kMaxBits = 16657, kMaxPrec = 64;
static const int32_t kMinExp = -1074;

static uint64_t hdr_mode(const gcow_params& p)
{
  const bool valid = p.minbits <= p.maxbits && p.maxprec >= 1 && p.maxprec <= 64;
  const bool dflt = p.minbits == kMinBits && p.maxbits == kMaxBits && p.maxprec == kMaxPrec && p.minexp == kMinExp;
  if (valid && !dflt) {
    if (p.minbits == p.maxbits && p.maxbits >= 1 && p.maxbits <= kMaxBits && p.maxprec >= kMaxPrec &&
        p.minexp <= kMinExp) {
      if (p.maxbits <= 2048) return p.maxbits - 1;
    } else if (p.minbits <= kMinBits && p.maxbits >= kMaxBits && p.minexp <= kMinExp) {
      if (p.maxprec <= 128) return (uint64_t)(p.maxprec - 1) + 2048;
    } else if (p.minbits <= kMinBits && p.maxbits >= kMaxBits && p.maxprec >= kMaxPrec && p.minexp >= kMinExp) {
      if (p.minexp <= 843) return (uint64_t)(p.minexp - kMinExp) + 2177;
    }
  }
  uint64_t m = (uint64_t)std::max(0, std::min(p.minexp + 16495, 0x7fff));
  m = (m << 7) + (std::max(1u, std::min(p.maxprec, 0x80u)) - 1);
  m = (m << 15) + (std::max(1u, std::min(p.maxbits, 0x8000u)) - 1);
  m = (m << 15) + (std::max(1u, std::min(p.minbits, 0x8000u)) - 1);
  return (m << 12) + 0xfffu;
}

static void put_bits(uint64_t* w, uint32_t& pos, uint64_t v, uint32_t n)
{
  if (n < 64) v &= (1ull << n) - 1ull;
  const uint32_t sh = pos & 63;
  w[pos >> 6] |= v << sh;
  if (sh && sh + n > 64) w[(pos >> 6) + 1] |= v >> (64 - sh);
  pos += n;
}

static uint64_t get_bits(const uint64_t* w, uint32_t& pos, uint32_t n)
{
  const uint32_t sh = pos & 63;
  uint64_t v = w[pos >> 6] >> sh;
  if (sh && sh + n > 64) v |= w[(pos >> 6) + 1] << (64 - sh);
  if (n < 64) v &= (1ull << n) - 1ull;
  pos += n;
  return v;
}

uint gcow_header_bits(const gcow_params* p) { return p && hdr_mode(*p) < 0xfffu ? 96u : 148u; }

uint gcow_write_header(const zfp_input* field, const gcow_params* p, uint64_t* words)
{
  const uint32_t d = dims_of(field);
  if (!p || !words || d < 1 || d > 4) return 0;
  const size_t n[4] = {field->nx, field->ny, field->nz, field->nw};
  const uint32_t w = d == 1 ? 48 : d == 2 ? 24 : d == 3 ? 16 : 12;
  for (uint32_t a = 0; a < d; a++)
    if (n[a] == 0 || (w < 64 && (uint64_t)(n[a] - 1) >> w)) return 0;
  uint64_t meta = 0;
  for (int a = (int)d - 1; a >= 0; a--) meta = (meta << w) + (uint64_t)(n[a] - 1);
  meta = (meta << 2) + (d - 1);
  meta = (meta << 2) + 2;  // zfp_type_float - 1
  words[0] = words[1] = words[2] = 0;
  uint32_t pos = 0;
  put_bits(words, pos, 0x0570667aull, 32);  // 'z' 'f' 'p' version 5
  put_bits(words, pos, meta, 52);
  const uint64_t mode = hdr_mode(*p);
  put_bits(words, pos, mode, mode < 0xfffu ? 12 : 64);
  return pos;
}

uint gcow_read_header(const uint64_t* words, size_t nwords, zfp_input* field, gcow_params* p)
{
  if (!words || !field || !p || nwords < 2) return 0;
  uint64_t w[3] = {words[0], words[1], nwords > 2 ? words[2] : 0};
  uint32_t pos = 0;
  if (get_bits(w, pos, 32) != 0x0570667aull) return 0;
  uint64_t meta = get_bits(w, pos, 52);
  if ((meta & 3u) + 1 != 3) return 0;  // float only
  meta >>= 2;
  const uint32_t d = (uint32_t)(meta & 3u) + 1;
  meta >>= 2;
  const uint32_t bw = d == 1 ? 48 : d == 2 ? 24 : d == 3 ? 16 : 12;
  size_t n[4] = {0, 0, 0, 0};
  for (uint32_t a = 0; a < d; a++) {
    n[a] = (size_t)(meta & ((1ull << bw) - 1)) + 1;
    meta >>= bw;
  }
  uint64_t mode = get_bits(w, pos, 12);
  gcow_params q{};
  if (mode < 0xfffu) {
    if (mode < 2048) {
      q = gcow_params{(uint)mode + 1, (uint)mode + 1, kMaxPrec, kMinExp};
    } else if (mode < 2048 + 128) {
      q = gcow_params{kMinBits, kMaxBits, (uint)mode + 1 - 2048, kMinExp};
    } else {
      q = gcow_params{kMinBits, kMaxBits, kMaxPrec, (int)mode + kMinExp - 2177};
    }
  } else {
    if (nwords < 3) return 0;
    mode = (mode + (get_bits(w, pos, 52) << 12)) >> 12;
    q.minbits = (uint)(mode & 0x7fffu) + 1;
    mode >>= 15;
    q.maxbits = (uint)(mode & 0x7fffu) + 1;
    mode >>= 15;
    q.maxprec = (uint)(mode & 0x7fu) + 1;
    mode >>= 7;
    q.minexp = (int)(mode & 0x7fffu) - 16495;
  }
  field->dtype = dtype_float;
  field->nx = n[0];
  field->ny = n[1];
  field->nz = n[2];
  field->nw = n[3];
  *p = q;
  return pos;
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

size_t gcow_encode_zfp_workspace_bytes(const zfp_input* field, const gcow_params* p)
{
  return align256(gcow_encode_workspace_bytes(field, p)) + 256 + align256(gcow_max_output_bytes(field, p));
}

gcow_status gcow_encode_device_zfp(const zfp_input* field, const gcow_params* p, void* d_out, size_t out_capacity,
                                   uint64_t* d_total_bits, void* d_workspace, size_t workspace_bytes,
                                   void* hip_stream)
{
  uint64_t h[3];
  const uint32_t hb = gcow_write_header(field, p, h);
  if (!hb) return fail(GCOW_ERR_INVALID, "field shape not representable in a zfp header (dims 1-4, 12 bits per axis in 4-D)");
  const size_t bound = gcow_max_output_bytes(field, p);
  if (!d_out || out_capacity < bound + 24) return fail(GCOW_ERR_CAPACITY, "output capacity below bound + 24");
  if (!d_workspace || workspace_bytes < gcow_encode_zfp_workspace_bytes(field, p))
    return fail(GCOW_ERR_INVALID, "workspace smaller than gcow_encode_zfp_workspace_bytes()");
  const size_t ews = gcow_encode_workspace_bytes(field, p);
  char* ws = (char*)d_workspace;
  uint64_t* d_bits = (uint64_t*)(ws + align256(ews));
  void* d_tmp = ws + align256(ews) + 256;
  gcow_status st = encode_impl(field, p, d_tmp, bound, d_bits, ews ? ws : nullptr, ews, nullptr, 0, hip_stream);
  if (st) return st;
  GCOW_HIP(gcow::launch_prepend_header((uint64_t*)d_out, hb, (const uint64_t*)d_tmp, d_bits, h,
                                       (uint64_t)(bound / 8) + 3, d_total_bits, hip_stream));
  return GCOW_OK;
}

gcow_status gcow_decode_device_at(const zfp_input* field, const gcow_params* p, const void* d_in, size_t in_bytes,
                                  uint64_t bit_offset, const uint64_t* d_index, uint32_t index_stride,
                                  void* hip_stream)
{
  return decode_impl(field, p, d_in, d_index, index_stride, bit_offset, nullptr, hip_stream, in_bytes);
}

gcow_status gcow_stitch_device(uint64_t* d_dst, uint64_t dst_bit_offset, const uint64_t* d_src, uint64_t src_bits,
                               void* hip_stream)
{
  if (!d_dst || (!d_src && src_bits)) return fail(GCOW_ERR_INVALID, "null stitch buffer");
  GCOW_HIP(gcow::launch_stitch(d_dst, dst_bit_offset, d_src, src_bits, hip_stream));
  return GCOW_OK;
}

gcow_status gcow_stitch_shards_device(uint64_t* d_dst, uint64_t dst_words, const uint64_t* d_src, uint64_t shard_words,
                                      const uint64_t* d_lens, uint32_t nshards, void* hip_stream)
{
  if (!d_dst && dst_words) return fail(GCOW_ERR_INVALID, "null destination");
  if (nshards && (!d_src || !d_lens)) return fail(GCOW_ERR_INVALID, "null shard buffer or lengths");
  GCOW_HIP(gcow::launch_stitch_shards(d_dst, dst_words, d_src, shard_words, d_lens, nshards, hip_stream));
  return GCOW_OK;
}

gcow_status gcow_decode_mean_device(const zfp_input* field, const gcow_params* p, const uint64_t* d_streams,
                                    size_t streams_bytes, uint64_t stream_words, uint32_t nstreams,
                                    const uint64_t* d_index, uint64_t index_words, uint32_t index_stride,
                                    void* hip_stream)
{
  gcow::FieldDesc F;
  gcow_status st = make_field(field, F, true, true);
  if (st) return st;
  if ((st = check_params(p, 1))) return st;
  if (F.dims != 1) return fail(GCOW_ERR_UNSUPPORTED, "decode_mean is for 1-D buckets");
  if (!nstreams || !d_streams) return fail(GCOW_ERR_INVALID, "no streams");
  // the decoders read up to two words past a stream's last bit (64-bit windows): the buffer holds them
  if (streams_bytes / 8 < (uint64_t)nstreams * stream_words + 2)
    return fail(GCOW_ERR_INVALID, "stream buffer smaller than nstreams * stream_words + 2 words");
  if (p->minbits != p->maxbits) {
    const uint32_t per = index_stride == GCOW_INDEX_PACKED16 ? 16u : index_stride;
    if (!d_index || (per != 8 && per != 16) || index_words < (F.nblocks + per - 1) / per)
      return fail(GCOW_ERR_INVALID, "variable-rate decode_mean needs each stream's index (stride 8 or 16, or packed16)");
  } else {
    if (d_index || index_stride || index_words)
      return fail(GCOW_ERR_INVALID, "fixed-rate decode_mean takes no block index (blocks are at b * maxbits)");
    if (stream_words < ((uint64_t)F.nblocks * p->maxbits + 63) / 64)
      return fail(GCOW_ERR_INVALID, "stream_words below one fixed-rate stream");
  }
  GCOW_HIP(gcow::launch_decode_mean1d(F, P(*p), d_streams, stream_words, nstreams, d_index, index_words, hip_stream,
                                      index_stride ? index_stride : 16));
  return GCOW_OK;
}

gcow_status gcow_index_pack16_device(const zfp_input* field, const gcow_params* p, const uint64_t* d_index8,
                                     uint64_t* d_out, void* hip_stream)
{
  if (!field || !p) return fail(GCOW_ERR_INVALID, "null field or params");
  if (get_input_dimension(field) != 1) return fail(GCOW_ERR_UNSUPPORTED, "packed16 index: 1-D fields only");
  gcow_status st = check_params(p, 1);
  if (st) return st;
  // a 1-D block codes at most 9 + 32 * 4 + 32 + 8 = 177 bits before minbits padding (header, four verbatim bits per
  // plane, one group flag per plane, the runs and flags of four coefficients turning significant)
  const uint64_t bmax = std::max<uint64_t>(p->minbits, std::min<uint64_t>(p->maxbits, 177));
  const uint64_t nb = get_input_num_blocks(field);
  if (8 * bmax > 0xffff || nb * bmax >= (1ull << 48))
    return fail(GCOW_ERR_UNSUPPORTED, "packed16 index: 8 blocks may exceed 65535 bits, or the stream 2^48 bits");
  const uint64_t n8 = (nb + 7) / 8;
  if (n8 && (!d_index8 || !d_out)) return fail(GCOW_ERR_INVALID, "null index buffer");
  GCOW_HIP(gcow::launch_index_pack16(d_index8, n8, d_out, hip_stream));
  return GCOW_OK;
}

gcow_status gcow_copy_pattern_device(const void* d_in, int dtype, size_t nvals, uint32_t out_bits_per_block,
                                     void* d_out, void* hip_stream)
{
  if ((!d_in || !d_out) && nvals >= 4) return fail(GCOW_ERR_INVALID, "null buffer");
  if (dtype != dtype_float && dtype != dtype_bf16) return fail(GCOW_ERR_UNSUPPORTED, "dtype_float or dtype_bf16");
  if (out_bits_per_block != 32 && out_bits_per_block != 64) return fail(GCOW_ERR_INVALID, "32 or 64 bits per block");
  if (nvals / 4 >= (1ull << 32)) return fail(GCOW_ERR_UNSUPPORTED, "more than 2^32 blocks per call");
  GCOW_HIP(gcow::launch_copy_pattern1d(d_in, dtype == dtype_bf16 ? gcow::DT_BF16 : gcow::DT_F32, nvals,
                                       out_bits_per_block, d_out, hip_stream));
  return GCOW_OK;
}

gcow_status gcow_debug_set_var1d_variant(int form, int spin, int stats)
{
  if (form < 0 || form > 2) return fail(GCOW_ERR_INVALID, "form: 0 tile, 1 range, 2 look-back single pass");
  gcow::g_var1d_variant = gcow::Var1dVariant{form, spin, stats};
  return GCOW_OK;
}

gcow_status gcow_fill_normal_device(float* d_out, size_t count, double sigma, uint64_t seed, int inject,
                                    void* hip_stream)
{
  if (!d_out && count) return fail(GCOW_ERR_INVALID, "null output");
  GCOW_HIP(gcow::launch_fill_normal(d_out, count, sigma, seed, inject, hip_stream));
  return GCOW_OK;
}

gcow_status gcow_stage_emax_device(const float* d_blocks, uint32_t nblocks, uint32_t dims, int32_t* d_emax,
                                   void* hip_stream)
{
  if (dims < 1 || dims > 3) return fail(GCOW_ERR_INVALID, "dims");
  GCOW_HIP(gcow::launch_stage(0, (int)dims, d_blocks, nullptr, nblocks, d_emax, 0, 0, nullptr, 0, hip_stream));
  return GCOW_OK;
}

gcow_status gcow_stage_cast_device(const float* d_blocks, const int32_t* d_emax, uint32_t nblocks, uint32_t dims,
                                   int32_t* d_iblocks, void* hip_stream)
{
  if (dims < 1 || dims > 3) return fail(GCOW_ERR_INVALID, "dims");
  GCOW_HIP(gcow::launch_stage(1, (int)dims, d_blocks, d_emax, nblocks, d_iblocks, 0, 0, nullptr, 0, hip_stream));
  return GCOW_OK;
}

gcow_status gcow_stage_xform_device(int32_t* d_iblocks, uint32_t nblocks, uint32_t dims, int inverse,
                                    void* hip_stream)
{
  if (dims < 1 || dims > 3) return fail(GCOW_ERR_INVALID, "dims");
  GCOW_HIP(gcow::launch_stage(2, (int)dims, nullptr, nullptr, nblocks, d_iblocks, (uint32_t)inverse, 0, nullptr, 0,
                              hip_stream));
  return GCOW_OK;
}

gcow_status gcow_stage_reorder_device(const int32_t* d_iblocks, uint32_t nblocks, uint32_t dims,
                                      uint32_t* d_ublocks, void* hip_stream)
{
  if (dims < 1 || dims > 3) return fail(GCOW_ERR_INVALID, "dims");
  GCOW_HIP(gcow::launch_stage(3, (int)dims, d_iblocks, nullptr, nblocks, d_ublocks, 0, 0, nullptr, 0, hip_stream));
  return GCOW_OK;
}

gcow_status gcow_stage_encode_ints_device(const uint32_t* d_ublocks, uint32_t nblocks, uint32_t dims,
                                          uint32_t budget, uint32_t maxprec, uint64_t* d_slots, uint32_t slot_words,
                                          uint32_t* d_bits, void* hip_stream)
{
  if (dims < 1 || dims > 3) return fail(GCOW_ERR_INVALID, "dims");
  if (slot_words < 4) return fail(GCOW_ERR_INVALID, "slot_words");
  GCOW_HIP(gcow::launch_stage(4, (int)dims, d_ublocks, nullptr, nblocks, d_slots, budget, maxprec, d_bits, slot_words,
                              hip_stream));
  return GCOW_OK;
}

// ================================================================================================ array codec
size_t zfp_compress(zfp_output* output, const zfp_input* input)
{
  // sw/src/zfp.c:10-28: encode every block, flush to a 64-bit boundary, return the stream size in bytes.
  stream* s = output->data;
  const uint32_t d = dims_of(input);
  const gcow_params p = params_of(output);
  gcow::FieldDesc F;
  if (d < 1 || d > 3 || make_field(input, F, false) != GCOW_OK || check_params(&p, d) != GCOW_OK) {
    stream_flush(s);  // unsupported input: no-op like sw/ (zfp.c:12-27)
    return stream_size_bytes(s);
  }
  OutState* st = state_of(output);
  st->valid = false;
  const uint64_t start = stream_woffset(s);
  const size_t esz = get_dtype_size(input->dtype);
  const size_t nvals = get_input_size(input, nullptr);
  const bool dev_in = is_device_ptr(input->data);
  const bool dev_out = is_device_ptr(s->begin);
  zfp_input in2 = *input;
  if (!dev_in) {
    // host input: stage it on the device. A strided array (sw/src/zfp.c:37-39, 45) is copied as the element span its
    // strides touch, and keeps its strides against the device copy.
    ptrdiff_t lo = 0, hi = (ptrdiff_t)nvals - 1;
    if (strided(input)) field_span(input, &lo, &hi);
    const size_t span = (size_t)(hi - lo + 1) * esz;
    if (grow(&st->d_data, &st->d_data_cap, span) != hipSuccess ||
        hipMemcpy(st->d_data, (const char*)input->data + lo * (ptrdiff_t)esz, span, hipMemcpyHostToDevice) !=
            hipSuccess) {
      g_err = "H2D copy failed";
      return 0;
    }
    in2.data = (char*)st->d_data - lo * (ptrdiff_t)esz;
  }
  const size_t cap = gcow_max_output_bytes(&in2, &p);
  const uint32_t stride = d == 3 ? 1 : (d == 2 ? 4 : 16);
  const size_t nidx = gcow_index_entries(&in2, stride);
  const size_t ws = gcow_encode_workspace_bytes(&in2, &p);
  if (grow(&st->d_stream, &st->d_stream_cap, cap) != hipSuccess ||
      grow((void**)&st->d_index, &st->d_index_cap, (nidx + 1) * 8) != hipSuccess ||
      grow(&st->d_ws, &st->d_ws_cap, ws + 8) != hipSuccess ||
      (!st->d_u64 && hipMalloc((void**)&st->d_u64, 24) != hipSuccess)) {
    g_err = "device allocation failed";
    return 0;
  }
  const bool fixed = p.minbits == p.maxbits;
  if (encode_impl(&in2, &p, st->d_stream, cap, st->d_u64, st->d_ws, ws, fixed ? nullptr : st->d_index, stride,
                  nullptr) != GCOW_OK)
    return 0;
  uint64_t bits = 0;
  if (hipMemcpy(&bits, st->d_u64, 8, hipMemcpyDeviceToHost) != hipSuccess) {
    g_err = "D2H copy failed";
    return 0;
  }
  const uint64_t words = (bits + 63) / 64;
  const uint64_t end_words = (start + bits + 63) / 64;
  if (s->end > 0 && end_words > (uint64_t)s->end) {
    g_err = "stream capacity exceeded";
    return 0;
  }
  if (start == 0 && s->buffered_bits == 0) {
    if (dev_out) {
      if (hipMemcpy(s->begin, st->d_stream, words * 8, hipMemcpyDeviceToDevice) != hipSuccess) return 0;
    } else if (hipMemcpy(s->begin, st->d_stream, words * 8, hipMemcpyDeviceToHost) != hipSuccess) {
      return 0;
    }
    s->idx = (ptrdiff_t)words;
    s->buffer = 0;
    s->buffered_bits = 0;
  } else {
    // appending after existing bits: move the stream through the host bit writer (stream.c semantics)
    uint64_t* tmp = (uint64_t*)malloc((words + 1) * 8);
    if (!tmp || hipMemcpy(tmp, st->d_stream, words * 8, hipMemcpyDeviceToHost) != hipSuccess) {
      free(tmp);
      return 0;
    }
    if (dev_out) {
      free(tmp);
      g_err = "appending to a device-resident stream is not supported";
      return 0;
    }
    append_bits(s, tmp, bits);
    free(tmp);
    stream_flush(s);
  }
  if (dev_out) {
    st->shadow.clear();
    st->shadow.shrink_to_fit();
  } else {
    st->shadow.assign((const uint64_t*)s->begin, (const uint64_t*)s->begin + words);
  }
  st->valid = true;
  st->host_begin = s->begin;
  st->words = words;
  st->bits = bits;
  st->index_stride = fixed ? 0 : stride;
  st->params = p;
  st->dims = d;
  st->nblocks = F.nblocks;
  if (start) st->valid = false;  // cached stream is not at offset 0 of the caller's stream
  return stream_size_bytes(s);
}

size_t zfp_decompress(zfp_output* output, const zfp_input* input)
{
  // sw/src/zfp.c:58-76 with libzfp block semantics: decode from the stream's read position, align to the next word.
  stream* s = output->data;
  const uint32_t d = dims_of(input);
  const gcow_params p = params_of(output);
  zfp_input in2 = *input;
  in2.dtype = dtype_float;
  gcow::FieldDesc F;
  if (d < 1 || d > 3 || input->dtype != dtype_float || make_field(&in2, F, true) != GCOW_OK ||
      check_params(&p, d) != GCOW_OK) {
    stream_algin_next_word(s);
    return stream_size_bytes(s);
  }
  OutState* st = state_of(output);
  const uint64_t start = stream_roffset(s);
  const size_t nvals = get_input_size(input, nullptr);
  const bool dev_out = is_device_ptr(input->data);
  const bool dev_stream = is_device_ptr(s->begin);
  const bool fixed = p.minbits == p.maxbits;
  bool cached = st->valid && start == 0 && st->host_begin == s->begin && st->dims == d &&
                st->nblocks == F.nblocks && std::memcmp(&st->params, &p, sizeof(p)) == 0;
  // the buffer must still hold the whole cached stream (a smaller buffer at the same address is not read past its end)
  if (cached && s->end > 0 && (uint64_t)s->end < st->words) cached = false;
  if (!st->d_u64 && hipMalloc((void**)&st->d_u64, 24) != hipSuccess) return 0;
  if (cached) {  // the caller may have rewritten its buffer since zfp_compress filled the cache: compare every word
    if (!dev_stream) {
      cached = st->shadow.size() == st->words &&
               std::memcmp(s->begin, st->shadow.data(), st->words * sizeof(uint64_t)) == 0;
    } else {
      uint64_t differ = 1;
      if (gcow::launch_words_differ((const uint64_t*)s->begin, (const uint64_t*)st->d_stream, st->words, st->d_u64 + 2,
                                    nullptr) != hipSuccess ||
          hipMemcpy(&differ, st->d_u64 + 2, 8, hipMemcpyDeviceToHost) != hipSuccess)
        return 0;
      cached = differ == 0;
    }
  }
  const void* d_stream;
  const uint64_t* d_index = nullptr;
  uint32_t stride = 0;
  uint64_t base = 0;
  if (cached) {
    d_stream = st->d_stream;
    d_index = fixed ? nullptr : st->d_index;
    stride = st->index_stride;
  } else {
    const uint64_t w0 = start / 64;
    const uint64_t avail = s->end > 0 ? (uint64_t)s->end - w0 : 0;
    const uint64_t need = std::min<uint64_t>(avail, (F.nblocks * block_bits_bound(p, d) + 127) / 64 + 2);
    if (grow(&st->d_stream, &st->d_stream_cap, (need + 2) * 8) != hipSuccess) return 0;
    st->valid = false;
    if (hipMemsetAsync(st->d_stream, 0, (need + 2) * 8, nullptr) != hipSuccess) return 0;
    const hipMemcpyKind k = dev_stream ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    if (need && hipMemcpy(st->d_stream, s->begin + w0, need * 8, k) != hipSuccess) return 0;
    d_stream = st->d_stream;
    base = start % 64;
  }
  // host output: decode into a device copy of the element span the strides touch (dense: the array itself), whose
  // untouched gaps are the caller's own values (sw/src/zfp.c:86-92 scatters through sx / sy)
  ptrdiff_t lo = 0, hi = (ptrdiff_t)nvals - 1;
  if (!dev_out && strided(input)) field_span(input, &lo, &hi);
  const size_t span = (size_t)(hi - lo + 1) * 4;
  if (!dev_out) {
    if (grow(&st->d_data, &st->d_data_cap, span) != hipSuccess) return 0;
    if (strided(input) && hipMemcpy(st->d_data, (const char*)input->data + lo * 4, span, hipMemcpyHostToDevice) !=
                              hipSuccess)
      return 0;
    in2.data = (char*)st->d_data - lo * 4;
  }
  if (decode_impl(&in2, &p, d_stream, d_index, stride, base, st->d_u64 + 1, nullptr) != GCOW_OK) return 0;
  uint64_t end = 0;
  if (fixed) {
    end = base + (uint64_t)F.nblocks * p.maxbits;
  } else if (hipMemcpy(&end, st->d_u64 + 1, 8, hipMemcpyDeviceToHost) != hipSuccess) {
    return 0;
  }
  if (!dev_out) {
    if (hipMemcpy((char*)input->data + lo * 4, st->d_data, span, hipMemcpyDeviceToHost) != hipSuccess) return 0;
  } else if (hipDeviceSynchronize() != hipSuccess) {
    return 0;
  }
  const uint64_t abs_end = start - base + end;
  stream_rseek(s, (abs_end + 63) / 64 * 64);  // stream_algin_next_word
  return stream_size_bytes(s);
}

// ================================================================================================ block API
// Gather / scatter are host data movement (sw/src/encode.c:41-126, decode.c:27-42); the numeric stages run on the
// GPU stage kernels through a small per-thread device scratch.
static void pad_partial_block(float* block, size_t n, ptrdiff_t s)
{
  switch (n) {
    case 0: block[0 * s] = 0; /* FALLTHROUGH */
    case 1: block[1 * s] = block[0 * s]; /* FALLTHROUGH */
    case 2: block[2 * s] = block[1 * s]; /* FALLTHROUGH */
    case 3: block[3 * s] = block[0 * s]; /* FALLTHROUGH */
    default: break;
  }
}

void gather_2d_block(float* block, const float* raw, ptrdiff_t sx, ptrdiff_t sy)
{
  for (size_t y = 0; y < 4; y++)
    for (size_t x = 0; x < 4; x++) block[4 * y + x] = raw[(ptrdiff_t)x * sx + (ptrdiff_t)y * sy];
}

void gather_partial_2d_block(float* block, const float* raw, size_t nx, size_t ny, ptrdiff_t sx, ptrdiff_t sy)
{
  for (size_t y = 0; y < ny; y++) {
    for (size_t x = 0; x < nx; x++) block[4 * y + x] = raw[(ptrdiff_t)x * sx + (ptrdiff_t)y * sy];
    pad_partial_block(block + 4 * y, nx, 1);
  }
  for (size_t x = 0; x < 4; x++) pad_partial_block(block + x, ny, 4);
}

void gather_4d_block(float* block, const float* raw, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz, ptrdiff_t sw)
{
  for (size_t w = 0; w < 4; w++)
    for (size_t z = 0; z < 4; z++)
      for (size_t y = 0; y < 4; y++)
        for (size_t x = 0; x < 4; x++)
          *block++ = raw[(ptrdiff_t)x * sx + (ptrdiff_t)y * sy + (ptrdiff_t)z * sz + (ptrdiff_t)w * sw];
}

void gather_partial_4d_block(float* block, const float* raw, size_t nx, size_t ny, size_t nz, size_t nw, ptrdiff_t sx,
                             ptrdiff_t sy, ptrdiff_t sz, ptrdiff_t sw)
{
  for (size_t w = 0; w < nw; w++) {
    for (size_t z = 0; z < nz; z++) {
      for (size_t y = 0; y < ny; y++) {
        for (size_t x = 0; x < nx; x++)
          block[64 * w + 16 * z + 4 * y + x] =
              raw[(ptrdiff_t)x * sx + (ptrdiff_t)y * sy + (ptrdiff_t)z * sz + (ptrdiff_t)w * sw];
        pad_partial_block(block + 64 * w + 16 * z + 4 * y, nx, 1);
      }
      for (size_t x = 0; x < 4; x++) pad_partial_block(block + 64 * w + 16 * z + x, ny, 4);
    }
    for (size_t y = 0; y < 4; y++)
      for (size_t x = 0; x < 4; x++) pad_partial_block(block + 64 * w + 4 * y + x, nz, 16);
  }
  for (size_t z = 0; z < 4; z++)
    for (size_t y = 0; y < 4; y++)
      for (size_t x = 0; x < 4; x++) pad_partial_block(block + 16 * z + 4 * y + x, nw, 64);
}

void scatter_2d_block(const float* block, float* raw, ptrdiff_t sx, ptrdiff_t sy)
{
  for (size_t y = 0; y < 4; y++)
    for (size_t x = 0; x < 4; x++) raw[(ptrdiff_t)x * sx + (ptrdiff_t)y * sy] = block[4 * y + x];
}

void scatter_partial_2d_block(const float* block, float* raw, size_t nx, size_t ny, ptrdiff_t sx, ptrdiff_t sy)
{
  for (size_t y = 0; y < ny; y++)
    for (size_t x = 0; x < nx; x++) raw[(ptrdiff_t)x * sx + (ptrdiff_t)y * sy] = block[4 * y + x];
}

int get_block_exponent(const float* block, uint n)
{
  // encode.c:142-152 on the GPU emax stage: 64-value chunks (zero padding never raises the max).
  const uint32_t chunks = (n + 63) / 64;
  float* h = (float*)calloc((size_t)chunks * 64, 4);
  int32_t* e = (int32_t*)malloc((size_t)chunks * 4);
  uint8_t* d = (uint8_t*)scratch((size_t)chunks * 64 * 4 + (size_t)chunks * 4);
  int r = -127;
  if (h && e && d) {
    std::memcpy(h, block, (size_t)n * 4);
    if (hipMemcpy(d, h, (size_t)chunks * 256, hipMemcpyHostToDevice) == hipSuccess &&
        gcow_stage_emax_device((const float*)d, chunks, 3, (int32_t*)(d + (size_t)chunks * 256), nullptr) == GCOW_OK &&
        hipMemcpy(e, d + (size_t)chunks * 256, (size_t)chunks * 4, hipMemcpyDeviceToHost) == hipSuccess)
      for (uint32_t i = 0; i < chunks; i++) r = e[i] > r ? e[i] : r;
  }
  free(h);
  free(e);
  return r;
}

int get_scaler_exponent(float x)
{
  // encode.c:128-140: only x > 0 has an exponent (negative and NaN inputs give -EBIAS)
  if (!(x > 0)) return -127;
  float b[4] = {x, 0, 0, 0};
  return get_block_exponent(b, 4);
}

void fwd_cast_block(int32* iblock, const float* fblock, uint n, int emax)
{
  // encode.c:178-187 on the GPU cast stage (64-value chunks, one emax each)
  const uint32_t chunks = (n + 63) / 64;
  float* h = (float*)calloc((size_t)chunks * 64, 4);
  int32_t* q = (int32_t*)malloc((size_t)chunks * 64 * 4);
  int32_t* em = (int32_t*)malloc((size_t)chunks * 4);
  uint8_t* d = (uint8_t*)scratch((size_t)chunks * (256 + 256 + 4));
  if (h && q && em && d) {
    std::memcpy(h, fblock, (size_t)n * 4);
    for (uint32_t i = 0; i < chunks; i++) em[i] = emax;
    float* df = (float*)d;
    int32_t* dq = (int32_t*)(d + (size_t)chunks * 256);
    int32_t* de = (int32_t*)(d + (size_t)chunks * 512);
    if (hipMemcpy(df, h, (size_t)chunks * 256, hipMemcpyHostToDevice) == hipSuccess &&
        hipMemcpy(de, em, (size_t)chunks * 4, hipMemcpyHostToDevice) == hipSuccess &&
        gcow_stage_cast_device(df, de, chunks, 3, dq, nullptr) == GCOW_OK &&
        hipMemcpy(q, dq, (size_t)chunks * 256, hipMemcpyDeviceToHost) == hipSuccess)
      std::memcpy(iblock, q, (size_t)n * 4);
  }
  free(h);
  free(q);
  free(em);
}

static bool xform_host(int32* iblock, uint32_t dims, int inverse)
{
  const size_t bytes = (size_t)4 << (2 * dims);
  int32_t* d = (int32_t*)scratch(bytes);
  return d && hipMemcpy(d, iblock, bytes, hipMemcpyHostToDevice) == hipSuccess &&
         gcow_stage_xform_device(d, 1, dims, inverse, nullptr) == GCOW_OK &&
         hipMemcpy(iblock, d, bytes, hipMemcpyDeviceToHost) == hipSuccess;
}

void fwd_decorrelate_2d_block(int32* iblock) { (void)xform_host(iblock, 2, 0); }

void fwd_reorder_int2uint(uint32* ublock, const int32* iblock, const uchar* perm, uint n)
{
  // encode.c:269-275 writes n + 1 values (one past the end); this writes exactly n. The permutation gather is host
  // data movement; the two's complement -> negabinary map runs on the GPU (identity-permuted 1-D stage, 4 at a time).
  const uint32_t chunks = (n + 3) / 4;
  int32_t* g = (int32_t*)calloc((size_t)chunks * 4, 4);
  uint32_t* u = (uint32_t*)malloc((size_t)chunks * 16);
  uint8_t* d = (uint8_t*)scratch((size_t)chunks * 32);
  if (g && u && d) {
    for (uint i = 0; i < n; i++) g[i] = iblock[perm[i]];
    if (hipMemcpy(d, g, (size_t)chunks * 16, hipMemcpyHostToDevice) == hipSuccess &&
        gcow_stage_reorder_device((const int32_t*)d, chunks, 1, (uint32_t*)(d + (size_t)chunks * 16), nullptr) ==
            GCOW_OK &&
        hipMemcpy(u, d + (size_t)chunks * 16, (size_t)chunks * 16, hipMemcpyDeviceToHost) == hipSuccess)
      std::memcpy(ublock, u, (size_t)n * 4);
  }
  free(g);
  free(u);
}

static uint dims_of_size(uint block_size) { return block_size == 4 ? 1 : (block_size == 16 ? 2 : (block_size == 64 ? 3 : 0)); }

static uint coder_host(stream* s, const uint32* ublock, uint budget, uint maxprec, uint block_size)
{
  const uint dims = dims_of_size(block_size);
  if (!dims) return 0;
  const uint32_t slot_words = 48;  // 3072 bits >= any 4^3 block
  uint8_t* d = (uint8_t*)scratch((size_t)block_size * 4 + slot_words * 8 + 8);
  if (!d) return 0;
  uint32_t* du = (uint32_t*)d;
  uint64_t* ds = (uint64_t*)(d + (size_t)block_size * 4);
  uint32_t* db = (uint32_t*)(ds + slot_words);
  uint64_t slot[48];
  uint32_t bits = 0;
  if (hipMemcpy(du, ublock, (size_t)block_size * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(ds, 0, slot_words * 8) != hipSuccess ||
      gcow_stage_encode_ints_device(du, 1, dims, budget, maxprec, ds, slot_words, db, nullptr) != GCOW_OK ||
      hipMemcpy(slot, ds, sizeof(slot), hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(&bits, db, 4, hipMemcpyDeviceToHost) != hipSuccess)
    return 0;
  append_bits(s, slot, bits);
  return bits;
}

uint encode_all_bitplanes(stream* const s, const uint32* const ublock, uint maxprec, uint block_size)
{
  return coder_host(s, ublock, 0xffffffffu, maxprec, block_size);  // encode.c:343-408
}

uint encode_partial_bitplanes(stream* const s, const uint32* const ublock, uint maxbits, uint maxprec,
                              uint block_size)
{
  return coder_host(s, ublock, maxbits, maxprec, block_size);  // encode.c:279-339
}

uint encode_iblock(stream* const out_data, uint minbits, uint maxbits, uint maxprec, int32* iblock, size_t dim)
{
  // encode.c:412-455, d-generic (sw/ only transforms 2-D and always uses PERM_2D)
  if (dim < 1 || dim > 3) return 0;
  const uint block_size = 1u << (2 * dim);
  if (!xform_host(iblock, (uint32_t)dim, 0)) return 0;
  uint32_t u[64];
  const size_t bytes = (size_t)block_size * 4;
  uint8_t* d = (uint8_t*)scratch(2 * bytes);
  if (!d || hipMemcpy(d, iblock, bytes, hipMemcpyHostToDevice) != hipSuccess ||
      gcow_stage_reorder_device((const int32_t*)d, 1, (uint32_t)dim, (uint32_t*)(d + bytes), nullptr) != GCOW_OK ||
      hipMemcpy(u, d + bytes, bytes, hipMemcpyDeviceToHost) != hipSuccess)
    return 0;
  const uint budget = exceeded_maxbits(maxbits, maxprec, block_size) ? maxbits : 0xffffffffu;
  uint bits = coder_host(out_data, u, budget, maxprec, block_size);
  if (bits < minbits) {
    stream_pad(out_data, minbits - bits);
    bits = minbits;
  }
  return bits;
}

uint encode_fblock(zfp_output* output, const float* fblock, size_t dim)
{
  // encode.c:457-495: one 4^d block through the full device encoder, appended to output->data.
  if (dim < 1 || dim > 3) return 0;
  const uint32_t B = 1u << (2 * dim);
  const gcow_params p = params_of(output);
  if (check_params(&p, (uint32_t)dim) != GCOW_OK) return 0;
  const uint64_t U = block_bits_bound(p, (uint32_t)dim);
  const size_t cap = (size_t)((U + 63) / 64 * 8 + 8);
  uint8_t* d = (uint8_t*)scratch((size_t)B * 4 + cap + 16);
  if (!d) return 0;
  float* df = (float*)d;
  uint64_t* dout = (uint64_t*)(d + (size_t)B * 4);
  uint64_t* dtot = (uint64_t*)(d + (size_t)B * 4 + cap);
  zfp_input f;
  std::memset(&f, 0, sizeof(f));
  f.dtype = dtype_float;
  f.data = df;
  f.nx = 4;
  f.ny = dim > 1 ? 4 : 0;
  f.nz = dim > 2 ? 4 : 0;
  uint64_t words[320];
  uint64_t bits = 0;
  const size_t ws = gcow_encode_workspace_bytes(&f, &p);
  uint64_t* wsp = nullptr;
  if (ws) {
    wsp = (uint64_t*)scratch((size_t)B * 4 + cap + 16 + ws);
    if (!wsp) return 0;
    d = (uint8_t*)wsp;
    df = (float*)d;
    dout = (uint64_t*)(d + (size_t)B * 4);
    dtot = (uint64_t*)(d + (size_t)B * 4 + cap);
    wsp = dtot + 2;
    f.data = df;
  }
  if (hipMemcpy(df, fblock, (size_t)B * 4, hipMemcpyHostToDevice) != hipSuccess ||
      encode_impl(&f, &p, dout, cap, dtot, wsp, ws, nullptr, 0, nullptr) != GCOW_OK ||
      hipMemcpy(&bits, dtot, 8, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(words, dout, (bits + 63) / 64 * 8, hipMemcpyDeviceToHost) != hipSuccess)
    return 0;
  append_bits(output->data, words, bits);
  return (uint)bits;
}

uint decode_fblock(zfp_output* output, float* fblock, size_t dim)
{
  // decode.c:220-253 with libzfp semantics: one block from the stream's read position.
  if (dim < 1 || dim > 3) return 0;
  const uint32_t B = 1u << (2 * dim);
  const gcow_params p = params_of(output);
  if (check_params(&p, (uint32_t)dim) != GCOW_OK) return 0;
  stream* s = output->data;
  const uint64_t start = stream_roffset(s);
  const uint64_t w0 = start / 64;
  const uint64_t U = block_bits_bound(p, (uint32_t)dim);
  uint64_t nw = (U + 127) / 64 + 1;
  if (s->end > 0 && w0 + nw > (uint64_t)s->end) nw = (uint64_t)s->end - w0;
  uint8_t* d = (uint8_t*)scratch((size_t)(nw + 2) * 8 + (size_t)B * 4 + 8);
  if (!d) return 0;
  uint64_t* dw = (uint64_t*)d;
  float* df = (float*)(d + (nw + 2) * 8);
  uint64_t* dend = (uint64_t*)(d + (nw + 2) * 8 + (size_t)B * 4);
  zfp_input f;
  std::memset(&f, 0, sizeof(f));
  f.dtype = dtype_float;
  f.data = df;
  f.nx = 4;
  f.ny = dim > 1 ? 4 : 0;
  f.nz = dim > 2 ? 4 : 0;
  uint64_t end = 0;
  if (hipMemset(dw, 0, (nw + 2) * 8) != hipSuccess ||
      hipMemcpy(dw, s->begin + w0, nw * 8, hipMemcpyHostToDevice) != hipSuccess)
    return 0;
  if (decode_impl(&f, &p, dw, nullptr, 0, start % 64, dend, nullptr) != GCOW_OK) return 0;
  if (p.minbits == p.maxbits) {
    end = start % 64 + p.maxbits;
  } else if (hipMemcpy(&end, dend, 8, hipMemcpyDeviceToHost) != hipSuccess) {
    return 0;
  }
  if (hipMemcpy(fblock, df, (size_t)B * 4, hipMemcpyDeviceToHost) != hipSuccess) return 0;
  const uint64_t bits = end - start % 64;
  stream_rseek(s, start + bits);
  return (uint)bits;
}

}  // extern "C"
