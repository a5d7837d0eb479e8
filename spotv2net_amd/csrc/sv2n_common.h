// Shared device helpers for the SpotV2Net MI355X kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include "sv2n.h"

#define SV2N_PSTR 36  // padded LDS row stride (floats) of a 32-wide attention row:
                      // 144 B keeps ds_read_b128 16-B aligned and spreads the
                      // transposed ds_write_b32 of a 32-lane half over 8 banks.

namespace sv2n {

enum Act { ACT_ID = 0, ACT_RELU = 1, ACT_TANH = 2, ACT_SIGMOID = 3 };

template <int ACT>
__device__ __forceinline__ float act_fwd(float z) {
  if constexpr (ACT == ACT_RELU) return z > 0.f ? z : 0.f;
  else if constexpr (ACT == ACT_TANH) return tanhf(z);
  else if constexpr (ACT == ACT_SIGMOID) return 1.f / (1.f + expf(-z));
  else return z;
}

// d act / d z expressed through the forward output y (torch's *_backward forms:
// relu: y>0, tanh: 1-y^2, sigmoid: y(1-y)).
template <int ACT>
__device__ __forceinline__ float act_bwd(float dy, float y) {
  if constexpr (ACT == ACT_RELU) return y > 0.f ? dy : 0.f;
  else if constexpr (ACT == ACT_TANH) return dy * (1.f - y * y);
  else if constexpr (ACT == ACT_SIGMOID) return dy * (1.f - y) * y;
  else return dy;
}

// quad (4-lane) butterflies through DPP quad_perm: lane^1 and lane^2.
__device__ __forceinline__ float dpp_xor1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float dpp_xor2(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
}

// reductions across one 32-lane half of the wave (a padded attention row)
__device__ __forceinline__ float red32_sum(float v) {
#pragma unroll
  for (int m = 16; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}
__device__ __forceinline__ float red32_max(float v) {
#pragma unroll
  for (int m = 16; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, 64));
  return v;
}

// Last-arriving workgroup of a launch (cdna_hip_programming.md §6 Guideline 16,
// counter form): every block publishes its plain-stored slab with an
// agent-scope release and takes a ticket; the block drawing nblocks-1 gets
// true (in all its threads) after an agent-scope acquire, so its plain loads
// see every block's slab.  It also resets the counter, which must be zero
// before the first launch.  s_flag: one int of the kernel's existing LDS.
__device__ __forceinline__ bool last_block_arrive(unsigned* cnt, unsigned nblocks, int* s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned tk = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = tk == nblocks - 1u;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *s_flag = last;
  }
  __syncthreads();
  return *s_flag != 0;
}

// Write-through hand-off (cdna_hip_programming.md §6 G16, the split-K recipe's
// "sc1 slab stores"): data handed to another workgroup of the launch is
// stored with st_sc1 (agent-scope relaxed atomic store = global_store sc1),
// every storing wave drains it (s_waitcnt vmcnt(0)) before the block's
// barrier, one lane takes a relaxed ticket, and the last arriver reads the
// data ONLY with ld_sc1.  No release / acquire fence: a fence in every block
// cost 3-4x the whole reduction here.
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool last_block_sc1(unsigned* cnt, unsigned nblocks, int* s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its sc1 stores are done
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned tk = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = tk == nblocks - 1u;
    if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_flag = last;
  }
  __syncthreads();
  return *s_flag != 0;
}

// Two-level tickets: same-address atomics serialise at L2 (a launch's blocks
// all finish together), so block b first takes a ticket on group counter
// b % 8, and only the last of each group on the top counter — ~nblocks/8 + 8
// serialised atomics instead of nblocks.  Counter words are SV2N_TICKET_STRIDE
// apart (their own 128-B lines): cnt[0] top, cnt[(1 + g) * stride] group g.
// All must be zero before the first launch; the last arrivers reset them.
#define SV2N_TICKET_STRIDE 32
static_assert(SV2N_TICKET_WORDS == 9 * SV2N_TICKET_STRIDE, "sv2n.h ticket size");
__device__ __forceinline__ bool ticket2_lane0(unsigned* cnt, unsigned nblocks) {
  const unsigned g = blockIdx.x & 7u;
  const unsigned groups = nblocks < 8u ? nblocks : 8u;
  const unsigned members = (nblocks - g + 7u) / 8u;
  unsigned* gc = cnt + (1 + g) * SV2N_TICKET_STRIDE;
  const unsigned tk = __hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (tk != members - 1u) return false;
  __hip_atomic_store(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned t2 = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t2 != groups - 1u) return false;
  __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}
// last_block_sc1 with two-level tickets (cnt: SV2N_TICKET_WORDS words)
__device__ __forceinline__ bool last_block_sc1_2(unsigned* cnt, unsigned nblocks, int* s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) *s_flag = ticket2_lane0(cnt, nblocks);
  __syncthreads();
  return *s_flag != 0;
}

// Two-level reduction in one launch: every block publishes its partial
// (st_sc1), the last block of group g = b % 8 sums its group's partials in
// block order into a group slab (st_sc1), and the last group finisher sums the
// group slabs in group order.  Deterministic; the serial tail reads nblocks/8
// + 8 partials per column instead of nblocks.
__device__ __forceinline__ bool group_last_sc1(unsigned* cnt, unsigned nblocks, int* s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g = blockIdx.x & 7u;
    const unsigned members = (nblocks - g + 7u) / 8u;
    unsigned* gc = cnt + (1 + g) * SV2N_TICKET_STRIDE;
    const unsigned tk = __hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = tk == members - 1u;
    if (last) __hip_atomic_store(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_flag = last;
  }
  __syncthreads();
  return *s_flag != 0;
}
__device__ __forceinline__ bool top_last_sc1(unsigned* cnt, unsigned nblocks, int* s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned groups = nblocks < 8u ? nblocks : 8u;
    const unsigned tk = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = tk == groups - 1u;
    if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_flag = last;
  }
  __syncthreads();
  return *s_flag != 0;
}

// Last-arriving workgroup WITHOUT publication: for when the last arriver
// reads nothing the others wrote and only needs "everyone is past this
// point" (e.g. a value every block read at its start may now be replaced).
// Relaxed ticket, no fences; the counter is reset by the last arriver.
__device__ __forceinline__ bool last_block_ticket(unsigned* cnt, unsigned nblocks, int* s_flag) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned tk = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = tk == nblocks - 1u;
    if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_flag = last;
  }
  __syncthreads();
  return *s_flag != 0;
}

// last_block_ticket with two-level tickets (cnt: SV2N_TICKET_WORDS words)
__device__ __forceinline__ bool last_block_ticket2(unsigned* cnt, unsigned nblocks, int* s_flag) {
  __syncthreads();
  if (threadIdx.x == 0) *s_flag = ticket2_lane0(cnt, nblocks);
  __syncthreads();
  return *s_flag != 0;
}

// Output head + MSE fused into the last layer's n <= 32 attention forward
// (sv2n_gat_attn_fwd_head_mse): w == nullptr: off.
struct HeadFuse {
  const float* w;       // [OC] GATModel.linear.weight (out_features 1)
  const float* b;       // [1] its bias, or NULL
  const float* target;  // [B·n]
  float* part;          // [B][OC + 2] per-graph partials: Σ dout·y per column, Σ dout, Σ diff²
  float inv_n2;         // 2 / (B·n): d mean((out - target)²) / d out
  float* gw;            // host side (k_head_fuse_finish): [OC] += Σ_g, or NULL
  float* gb;            // [1] += Σ_g, or NULL
  float* loss;          // [1] = mean((out - target)²)
  float* loss_sum;      // [1] += loss, or NULL (a running sum the caller keeps)
};

// Edge-gradient tail of the n <= 32 attention backward (sv2n_attn_canon.hip,
// sv2n_gat_attn_bwd_edge): the edge pass's hl_pad columns it carries, and its
// arguments (ea == nullptr: off).
constexpr int ET_COLS = 8;
struct EdgeTail {
  const float* ea;                     // [B·E0][D] edge_attr (canonical order)
  const float* dae[SV2N_MAX_LAYERS];   // other layers' d-logits [B·E0][H] (own: unused)
  float* part;                         // [B][D][hlp] per-graph partials
  int D, L, own, hlp;                  // own: this layer's index (columns own·H ..)
};

// rows i of graph g: bit j set <=> edge j->i present (self loop excluded)
__device__ __forceinline__ uint32_t row_bits(const uint32_t* rowmask, int64_t row, int n, int i) {
  if (rowmask) return rowmask[row] & ~(1u << i);
  const uint32_t all = (n >= 32) ? 0xffffffffu : ((1u << n) - 1u);
  return all & ~(1u << i);
}

// edge e -> (graph g, target i, source j); false for self loops / out-of-block
// Canonical edge e of an n-node graph (CovarianceLaggedDataset order,
// reference utils/dataset.py:216-226: the P = n(n-1)/2 row-major upper pairs
// (u, w) as u -> w, then the same pairs swapped) -> (target i, source j),
// without a table: the pair index p inverts tri_off(n, u) = u(2n-u-1)/2.
__device__ __forceinline__ void canon_decode(int e, int n, int& i, int& j) {
  const int P = n * (n - 1) / 2;
  const bool lo = e >= P;
  const int p = lo ? e - P : e;
  const float b = 2.f * (float)n - 1.f;
  int u = (int)((b - sqrtf(fmaxf(b * b - 8.f * (float)p, 0.f))) * 0.5f);
  u = max(0, min(u, n - 2));
  while (u < n - 2 && (u + 1) * (2 * n - u - 2) / 2 <= p) ++u;
  while (u > 0 && u * (2 * n - u - 1) / 2 > p) --u;
  const int w = u + 1 + (p - u * (2 * n - u - 1) / 2);
  i = lo ? u : w;
  j = lo ? w : u;
}
// the canonical edge after (i, j): advances the pair state (lo, u, w)
struct CanonIt {
  int lo, u, w;
  __device__ __forceinline__ void init(int e, int n) {
    const int P = n * (n - 1) / 2;
    int i, j;
    canon_decode(e, n, i, j);
    lo = e >= P;
    u = lo ? i : j;
    w = lo ? j : i;
  }
  __device__ __forceinline__ void next(int n) {
    if (++w == n) {
      ++u;
      w = u + 1;
      if (u == n - 1) { lo ^= 1; u = 0; w = 1; }
    }
  }
  __device__ __forceinline__ int i() const { return lo ? u : w; }
  __device__ __forceinline__ int j() const { return lo ? w : u; }
};

__device__ __forceinline__ bool decode_edge(int64_t e, const int64_t* __restrict__ ei, int64_t E,
                                            const uint16_t* __restrict__ canon, int E0, int n,
                                            int64_t B, int64_t& g, int& i, int& j) {
  if (ei) {
    const int64_t s = ei[e], t = ei[E + e];
    if (s == t) return false;
    g = t / n;
    i = (int)(t - g * n);
    const int64_t jj = s - g * n;
    if (jj < 0 || jj >= n || g >= B || g < 0) return false;
    j = (int)jj;
    return true;
  }
  g = e / E0;
  const uint16_t c = canon[e - g * E0];
  i = c >> 8;
  j = c & 0xFF;
  return g < B;
}

// ---- buffer descriptors (cdna_hip_programming.md T8/T20) -------------------
// A raw buffer over [base, base + bytes): loads at an offset past `bytes`
// return 0 and stores there are dropped by the hardware, so predicated
// accesses need no branch and the compiler can count vmcnt across them.
// Build descriptors only from wave-uniform values (kernel args, blockIdx);
// `bytes` = 0 makes every access through the descriptor a no-op.
// Diagnostic bound checks (make CHECK=1; tests/conftest.py checks the count
// after every test when the library exports sv2n_check_hits).  SV2N_CHK
// compares a plain-pointer global index with its allocation's extent and
// COUNTS a violation (one device word per translation unit, plus the first
// failing site id) instead of dereferencing it; buffer loads and stores need
// no check (the descriptor bounds them).  Release builds compile it away.
#ifdef SV2N_CHECK
static __device__ unsigned int sv2n_chk_hits[2];
__device__ __noinline__ void sv2n_chk_fail(unsigned site) {
  if (__hip_atomic_fetch_add(&sv2n_chk_hits[0], 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT) == 0u)
    __hip_atomic_store(&sv2n_chk_hits[1], site, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
#define SV2N_CHK(site, idx, extent)                                              \
  do {                                                                           \
    if ((uint64_t)(int64_t)(idx) >= (uint64_t)(int64_t)(extent)) sv2n_chk_fail(site); \
  } while (0)
#define SV2N_CHK_EXPORT(tu)                                                      \
  extern "C" unsigned sv2n_check_hits_##tu(unsigned* first) {                    \
    unsigned h[2] = {0u, 0u};                                                    \
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(sv2n::sv2n_chk_hits), sizeof(h));        \
    const unsigned z[2] = {0u, 0u};                                              \
    (void)hipMemcpyToSymbol(HIP_SYMBOL(sv2n::sv2n_chk_hits), z, sizeof(z));        \
    if (first && h[0]) *first = h[1];                                            \
    return h[0];                                                                 \
  }
#else
#define SV2N_CHK(site, idx, extent) ((void)0)
#define SV2N_CHK_EXPORT(tu)
#endif

// The wave's index in its workgroup as a wave-uniform (SGPR) value.  threadIdx.x
// >> 6 is uniform in fact, but the compiler cannot prove it, and a buffer
// descriptor or soffset derived from it would then be made uniform lane by
// lane around every buffer instruction (a v_readfirstlane waterfall loop per
// load; tools/isa_waterfall.py finds them).
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int OOB = 0x7ffffff0;  // byte offset past any buffer (< 2^31)

// Every descriptor in this library is wave-uniform by construction (bases and
// sizes from block, graph and wave indices).  Values the compiler computed on
// the vector ALU (e.g. a runtime division of blockIdx.x) would otherwise give
// a waterfall loop around every buffer instruction that uses the descriptor:
// the base and size go through v_readfirstlane here.  Never build a descriptor
// from a per-lane value.
// The compiler folds __builtin_amdgcn_readfirstlane of a value it knows to be
// uniform, even one it keeps in a VGPR: an empty asm makes the value opaque
// first.  (The readfirstlane itself stays the builtin, so the hazard
// recognizer sees it and keeps the wait states between a VALU write of an
// SGPR and a memory instruction reading that SGPR; a readfirstlane written as
// inline asm does not get them.)
__device__ __forceinline__ uint32_t to_sgpr(uint32_t v) {
  asm volatile("" : "+v"(v));
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  const uint64_t b = reinterpret_cast<uint64_t>(base);
  const uint64_t lo = to_sgpr((uint32_t)b), hi = to_sgpr((uint32_t)(b >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((hi << 32) | lo), (short)0,
                                           (int)to_sgpr(bytes), 0x00020000);
}
// (the b32/b128 builtins move raw bits: unsigned int / uint x4)
__device__ __forceinline__ uint32_t bld_u32(rsrc_t r, int off) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
}
__device__ __forceinline__ float bld(rsrc_t r, int off) { return __uint_as_float(bld_u32(r, off)); }
__device__ __forceinline__ f32x4 bld4(rsrc_t r, int off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ u32x4 bld4_u32(rsrc_t r, int off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u32x2 bld2_u32(rsrc_t r, int off) {
  return __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
}
__device__ __forceinline__ void bst(rsrc_t r, int off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, 0);
}
__device__ __forceinline__ void bst2(rsrc_t r, int off, float a, float b) {
  __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(a), __float_as_uint(b)}, r, off, 0,
                                        0);
}
__device__ __forceinline__ void bst4(rsrc_t r, int off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, 0);
}

}  // namespace sv2n
