// engine.hip — batched PV-MCTS + self-play for MI355X (gfx950, wave64).
//
// Many independent PUCT trees live in flat pools in HBM, one 16-byte record per
// node: {W f32 value sum, P f32 prior, meta (visits N : 16 | action : 7 | |legal| : 7
// | 2 flags), link (first child : 20 | k copies : 12)}, indexed t * cap + local, the
// root at local 0. A node's children are one contiguous block of k*|legal| records
// (k = copies of the flushed leaf, uttt_mcts.cpp:121-135 + :38-43 append semantics),
// so the PUCT scan reads one 16-byte record per child, fully coalesced. States are never stored per node: a descent replays
// the actions from the root on bitboards (uttt_bits.h).
//
// One round (uttt_mcts.cpp:109-167, all trees in lock-step):
//   k_select  one wave per tree: descend by PUCT (wave arg-max, first index
//             wins ties), back up terminal simulations in place, stop at the
//             first unexpanded leaf -> pending record (node, path, k).
//   k_scan    one block: pending flags -> dense slots in tree order.
//   k_encode  one thread per input element: leaf -> NCHW (3,9,9) f32 row.
//   (evaluator: DualNetwork under PyTorch-ROCm, or k_hash_eval)
//   k_apply   one wave per pending leaf: legal-mask + sequential f32
//             renormalisation, k child blocks, k back-ups along the path.
// Self-play (self_play_cpp.py) adds k_move_end (scores, f64 policy target,
// numpy-legacy MT19937 choice, records), k_finalize (refill + arena offsets)
// and k_archive.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "uttt_bits.h"
#include "uttt_engine.h"

namespace uttt {

// ------------------------------------------------------------------ errors --
void set_error(const char *fmt, ...);  // rules_api.cpp (uttt_last_error)

#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess) {                                                              \
            set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
            return UTTT_ERR_HIP;                                                             \
        }                                                                                    \
    } while (0)

// ------------------------------------------------------------------ layout --
constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;
constexpr int kMaxDepth = 128;  // path slots: lane d holds path[d] and path[64 + d]
constexpr int kMaxPlies = 81;   // a game fills at most every cell
constexpr int kNone = 0x7fffffff;

constexpr int32_t kLive = 1;
constexpr int32_t kErrCapacity = 2;
constexpr int32_t kErrDepth = 4;
constexpr int32_t kErrSelect = 8;
constexpr int32_t kErrNonFinite = 16;  // the evaluator returned a NaN / Inf legal prior or value
constexpr int32_t kErrMask = kErrCapacity | kErrDepth | kErrSelect | kErrNonFinite;

// a failed tree's status -> message and UTTT_ERR_* (the checks that raise it are at the move / search end)
static const char *tree_error_text(uint32_t st) {
    return (st & kErrCapacity)    ? "node pool exhausted"
           : (st & kErrDepth)     ? "path deeper than 128"
           : (st & kErrNonFinite) ? "non-finite evaluator output (NaN or Inf in a legal prior or the value)"
                                  : "no selectable child (NaN statistics)";
}
static int tree_error_code(uint32_t st) {
    return (st & kErrCapacity) || (st & kErrDepth) ? UTTT_ERR_CAPACITY
           : (st & kErrNonFinite)                  ? UTTT_ERR_NONFINITE
                                                   : UTTT_ERR_ARG;
}

enum KernelId {
    kKSelect = 0, kKApply, kKEncode, kKScan, kKMoveEnd, kKHash,
    // select latency telemetry (counters only, no launches): dependent tree levels walked
    // (sum over trees of sum over descents of depth + 1), trees that descended, the current
    // launch's slowest tree (folded into the sum by k_scan after every select), that sum
    kKSelLevels, kKSelTrees, kKSelMax, kKSelMaxSum,
    // dependent memory round trips (the latency model's unit): sum over trees, the current launch's
    // slowest tree, that slowest count summed over launches
    kKSelTrips, kKSelTripMax, kKSelTripMaxSum,
    // the slowest-tree rows of odd rounds in uttt_rounds_hash_move's per-block form (k_round1 with part_host):
    // each round folds the previous round's rows at its start, so no round needs a last block
    kKSelMaxB, kKSelTripMaxB, kKernelCount
};

// Device counters are striped: counter i of a row lives in kStripes 128-byte slots, and a workgroup
// adds into slot (blockIdx & (kStripes - 1)), so thousands of waves finishing together do not
// serialize on one address (the host sums the slots).
constexpr int kStripes = 32;
constexpr int kStripeStride = 16;  // u64 per slot: 128 B
constexpr int kRow = kStripes * kStripeStride;  // u64 per counter
__device__ __forceinline__ unsigned long long *stripe_of(unsigned long long *row) {
    return row + (size_t)(blockIdx.x & (kStripes - 1)) * kStripeStride;
}

struct TreeCtl {
    int32_t sims_done;
    int32_t node_count;
    int32_t status;
    int32_t pad;
};

struct LeafRec {
    int32_t node;
    int32_t depth;
    int32_t k;
    int32_t pad;
};

// A single-tree search's round result in fine-grained pinned host memory (round 5, uttt_search_select_host):
// k_scan stores the counts, the pending leaf's state and its copies, then the tag (a system-scope release),
// and the host polls the tag: one select per flush costs no copy operation and no stream synchronisation
// (the reference's flush loop, uttt_mcts.cpp:109-167, runs in-process).
struct HostLeaf {
    int32_t count, stopped, left, tag;
    int32_t k, pad0, pad1, pad2;
    uttt_state_t state;
};

// One node (round 4: four SoA arrays N, W, P, LINK became one record, so the PUCT scan loads a child
// with one dwordx4 and an expansion stores a child with one):
//   .x W (f32 bits)   .y P (f32 bits)
//   .z meta: visits N (bits 0-15) | action (16-22) | L = |legal| of the node's state, the size of
//      each of its child blocks (23-29) | kMetaP64 (30) | kMetaWF32 (31)
//   .w link: first child (bits 0-19) | k = its child blocks (20-31)
// Limits: max_sims <= 4095 (k and N fit; the pool cap 82 + 81 * max_sims < 2^20 first-child indices).
struct Pool {
    uint4 *rec;
    int64_t cap;
};
constexpr int kMaxSimsRec = UTTT_MAX_SIMS;
static_assert(82 + 81ll * kMaxSimsRec < (1ll << 20), "first-child index: 20 bits");
constexpr int kCountRing = 8;  // host-visible count slots per engine (uttt_search_select_async_to)

struct Trees {
    TreeCtl *ctl;
    uttt_state_t *root;
    uttt_state_t *leaf;
    LeafRec *rec;
    int32_t *path;    // [tree][kMaxDepth]
    uint4 *path_rec;  // [tree][kMaxDepth]: the path nodes' records as the select read them (k_apply's back-up
                      // starts from them instead of re-reading each node: one dependent round trip less)
    int32_t *pending; // [tree]: 0 nothing, 2 stopped by the select budget, 1 / 3 a queued leaf (3: the
                      // tree has simulations left after it) | the leaf's depth << 8
    int32_t *tree_of; // [slot]
    int32_t *depth_of; // [slot]: the queued leaf's depth (k_apply loads only the path entries it uses)
    int32_t *slot_of;  // [tree]: its queued leaf's slot this round, -1 for none (k_round: apply by tree)
    int32_t *count;   // [0] pending leaves this round, [1] trees stopped by the select budget,
                      // [2] trees with simulations left after this round's apply
    int32_t n_trees;
    int32_t sims;
    int32_t batch;
    int32_t py;  // 1: pv_mcts.py semantics (arena), 0: cpp/uttt_mcts.cpp (self-play)
    int32_t budget;  // in-place completions per tree and select launch (kSelectBudget; UTTT_SELECT_BUDGET)
};
// count[3]: nonzero once any tree of the search has failed (reset by k_begin): the asynchronous move end reads
// it instead of a launch that scans every tree's status (k_finalize finds the first failed tree only then)
__device__ __forceinline__ void flag_tree_error(const Trees &tr) { atomicOr(tr.count + 3, 1); }

// record packing (Pool)
constexpr uint32_t kNoAction = 0x7Fu;
__host__ __device__ __forceinline__ uint32_t make_meta(uint32_t action, uint32_t L) {  // N = 0
    return ((action & 0x7Fu) << 16) | ((L & 0x7Fu) << 23);
}
__host__ __device__ __forceinline__ int meta_n(uint32_t m) { return (int)(m & 0xFFFFu); }
__host__ __device__ __forceinline__ int meta_action(uint32_t m) { return (int)((m >> 16) & 0x7Fu); }
__host__ __device__ __forceinline__ int meta_L(uint32_t m) { return (int)((m >> 23) & 0x7Fu); }
// py semantics only (pv_mcts.py, NumPy 2 scalar promotion):
constexpr uint32_t kMetaP64 = 1u << 30;   // this node's children carry float64 uniform priors
constexpr uint32_t kMetaWF32 = 1u << 31;  // this node's w has become np.float32 (a network value)
constexpr uint32_t kMetaLMask = 0x7Fu << 23;
__host__ __device__ __forceinline__ uint32_t make_link(uint32_t first, uint32_t k) { return (first & 0xFFFFFu) | (k << 20); }
__host__ __device__ __forceinline__ int link_first(uint32_t l) { return (int)(l & 0xFFFFFu); }
__host__ __device__ __forceinline__ int link_k(uint32_t l) { return (int)(l >> 20); }
__device__ __forceinline__ uint4 new_child(float p, uint32_t action) {
    return make_uint4(0u, __float_as_uint(p), make_meta(action, 0u), 0u);
}

// ------------------------------------------------------------ wave helpers --
__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & (kWave - 1)); }
// This wave's global index (one wave per tree / slot / row), marked wave-uniform: what is derived from
// it (the tree's control words, its states, the rules applied to them) lives in scalar registers and
// runs on the scalar unit instead of as 64 identical vector lanes (round 4)
__device__ __forceinline__ int wave_index() {
    return __builtin_amdgcn_readfirstlane((int)(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)));
}

__device__ __forceinline__ uint64_t lanes_below() {
    const int l = lane_id();
    return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// Wave-wide arg-max: larger value wins, equal values -> smaller index
// (the reference's strict '>' scan in child order, uttt_mcts.cpp:69-78).
__device__ __forceinline__ void wave_argmax_d(double &v, int &i) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const double ov = __shfl_xor(v, off);
        const int oi = __shfl_xor(i, off);
        if (ov > v || (ov == v && oi < i)) {
            v = ov;
            i = oi;
        }
    }
}

__device__ __forceinline__ float readlane_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// The same arg-max by DPP lane moves, no LDS round trips (k_select's per-level reduction): the wave's
// largest value by one reduction of one instruction pair per step, then the smallest index among the
// lanes holding it ("larger value, then smaller index": the reference's strict '>' scan in child order)
// from one ballot when the maximum is unique, else from per-group ballots. Values are never NaN here (the per-lane scan's strict '>' from -1e9 never takes one); -0 and
// +0 compare equal, so they tie on the index as in the scan. Each reduction runs within each row of 16
// lanes (quad swaps, half-row and row mirrors), then row 0 into row 1 and row 2 into row 3
// (row_bcast15), then row 1 into rows 2-3 (row_bcast31): the result is valid in lane 63.
// one reduction step as a single DPP-sourced VALU op (the two wait states a DPP read of a VGPR
// written by the previous VALU op needs are in the asm: the compiler does not see inside it)
#define UTTT_DPP_STEP(op, ctl)                                                                     \
    __device__ __forceinline__ void op##_##ctl(uint32_t &k) {                                      \
        asm volatile("s_nop 1\n\t" #op "_dpp %0, %0, %0 " UTTT_DPP_##ctl : "+v"(k));             \
    }
#define UTTT_DPP_q1 "quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
#define UTTT_DPP_q2 "quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf"
#define UTTT_DPP_hm "row_half_mirror row_mask:0xf bank_mask:0xf"
#define UTTT_DPP_rm "row_mirror row_mask:0xf bank_mask:0xf"
#define UTTT_DPP_b15 "row_bcast:15 row_mask:0xa bank_mask:0xf"
#define UTTT_DPP_b31 "row_bcast:31 row_mask:0xc bank_mask:0xf"
UTTT_DPP_STEP(v_max_u32, q1)
UTTT_DPP_STEP(v_max_u32, q2)
UTTT_DPP_STEP(v_max_u32, hm)
UTTT_DPP_STEP(v_max_u32, rm)
UTTT_DPP_STEP(v_max_u32, b15)
UTTT_DPP_STEP(v_max_u32, b31)
// wave-uniform result: the index of the largest v, the lowest index among equal maxima
// (cnt: the scanned child count; candidate indices are below it)
__device__ __forceinline__ int wave_argmax(float v, int i, int cnt) {
    // the value as an order-preserving unsigned (-0 canonicalised to +0 first), so each step of the max
    // is an integer max (no float canonicalisation)
    uint32_t b = __float_as_uint(v + 0.0f);
    b = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
    uint32_t m = b;
    v_max_u32_q1(m);   // quad_perm [1,0,3,2]
    v_max_u32_q2(m);   // quad_perm [2,3,0,1]
    v_max_u32_hm(m);   // row_half_mirror
    v_max_u32_rm(m);   // row_mirror
    v_max_u32_b15(m);  // row_bcast15 -> rows 1, 3
    v_max_u32_b31(m);  // row_bcast31 -> rows 2, 3
    asm volatile("s_nop 1");  // the asm's VALU write before the compiler's reads of m
    const uint32_t top = (uint32_t)__builtin_amdgcn_readlane((int)m, 63);
    // the usual case: one lane holds the maximum, and its index is the answer (no second pass)
    const uint64_t at = __ballot(b == top);
    if (__popcll(at) == 1) return __builtin_amdgcn_readlane(i, __builtin_ctzll(at));
    // ties (a node expanded by a flush of k copies holds k equal children per action until they are
    // visited): the smallest index among the lanes holding the maximum. Lane l's candidate is its own first
    // maximum, child l + 64 g of its scan group g (i & 63 == l), so the answer is the lowest such lane of
    // the lowest group present: one ballot per group from group 0 (round 5: in place of a second 6-step DPP
    // reduction and its wait states; usually group 0 or 1 answers). Every scan group of the node is
    // covered: a flush of k copies gives up to k x 81 children, more than 64 groups past batch 50.
    const int ngroups = (cnt + kWave - 1) / kWave;
    for (int g = 0; g < ngroups; ++g) {
        const uint64_t m = __ballot(b == top && (i >> 6) == g);
        if (m) return g * kWave + __builtin_ctzll(m);
    }
    return kNone;  // unreachable: some lane holds the maximum with a child index
}

// Orders this wave's global stores before its later global loads (other lanes
// read what one lane wrote; same CU, so workgroup scope suffices).
__device__ __forceinline__ void wave_memory_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

// Stores to host-visible (fine-grained pinned) words: system-coherent (sc0 sc1) and relaxed. A hand-off to
// the host is these stores, one s_waitcnt vmcnt(0) (they are acknowledged), then the tag, also relaxed: no
// release fence, whose L2 write-back (buffer_wbl2 sc0 sc1) would flush every line the kernel dirtied in the
// XCD's L2 (tree records, rows) to HBM at each hand-off, when the host reads only these words (round 6)
__device__ __forceinline__ void st_host(int32_t *a, int32_t v) {
    __hip_atomic_store(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_host(float *a, float v) {
    __hip_atomic_store(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void host_stores_done() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ------------------------------------------------------ evaluation cache --
// Open-addressing table in HBM: position (32 B) -> raw evaluator output (81
// priors + value, before legal masking). The evaluator is a pure function of
// the position (the reference feeds it to_input_tensor(), uttt_game.cpp:244),
// so a hit replays exactly what a new evaluation would return. Looked up in
// k_select (a hit is expanded in place: no network round), filled by k_apply.
constexpr int kProbe = 8;
constexpr int kCacheVal = 82;
// One record per slot, three 128-byte lines: the key (32 B), the 82 values (328 B), padding. Written
// and read as 16-byte agent-scope (sc1) accesses, 23 lanes of one wave: one fabric write per 16 B
// instead of one per 4-byte store (MI355X_MICROARCH.md: narrow sc1 stores are one fabric write each).
constexpr int kRecBytes = 384;
constexpr int kRecVal = 32;  // the key is the record's first 32 bytes
constexpr int kRecLanes = 23;  // 16-byte pieces written per record: 2 of key, 21 of values
constexpr int kSc1 = 16;       // buffer-intrinsic cache-policy bit: sc1 (agent scope)
static_assert(kRecVal + 16 * (kRecLanes - 2) >= kRecVal + 4 * kCacheVal && 16 * kRecLanes <= kRecBytes, "record");

struct EvalCache {
    // Per slot one flag word: bits 0-15 a version (0 empty; odd: a writer holds the slot; even >= 2:
    // ready), bits 16-31 the ready entry's tag (16 bits of its position's hash). A writer claims by
    // CAS from the value it saw to that + 1 and publishes the version + 2 with the new tag, so every
    // publish is a new flag value: a reader compares the flag it probed with the flag after its copy
    // (a seqlock without ABA). Probes read only the flags (32 contiguous bytes for 8 slots) and
    // load a record only for a ready slot whose tag matches (round 4: rounds 1-3 read 8 keys per probe).
    uint32_t *flag;
    char *rec;           // [slot][kRecBytes]
    uint32_t mask;       // capacity - 1
    unsigned long long *ctr;  // [0] hits, [1] misses (network leaves), [2] inserts, [3] replacements
};

__device__ __forceinline__ bool flag_ready(uint32_t f) { return (f & 0xFFFFu) != 0u && !(f & 1u); }
__device__ __forceinline__ uint32_t flag_tag(uint32_t f) { return f >> 16; }
// the flag that publishes a slot claimed from flag f (f & 0xFFFF even, or 0 for an empty slot)
__device__ __forceinline__ uint32_t flag_publish(uint32_t f, uint32_t tag) {
    const uint32_t v = (f & 0xFFFFu) + 2u;
    return (tag << 16) | (v > 0xFFFFu ? 2u : v);
}

__device__ __forceinline__ uint64_t state_hash64(const uttt_state_t &s) {
    const uint64_t a = ((uint64_t)s.own[1] << 32) | s.own[0];
    const uint64_t b = ((uint64_t)s.opp[0] << 32) | s.own[2];
    const uint64_t c = ((uint64_t)s.opp[2] << 32) | s.opp[1];
    const uint64_t d = ((uint64_t)(uint32_t)s.active << 32) | s.mains;
    return mix64(mix64(mix64(mix64(kGold ^ a) ^ b) ^ c) ^ d);
}
// a position's tag: the top 16 bits of its hash (its slot: the low 32 bits)
__device__ __forceinline__ uint32_t state_tag(uint64_t h64) { return (uint32_t)(h64 >> 48); }

// 16-byte piece `hi` (0 or 1) of a position's 32-byte key, by selects: indexing the state's words by a
// lane-dependent offset made the state a private array, which the compiler placed in LDS addressed by
// the flat work-item id, i.e. a read of the dispatch packet in host memory at every launch (round 4:
// 2-26 us before k_select's first descent, tools/diag/select_cycles.py)
__device__ __forceinline__ uint4 key_piece(const uttt_state_t &s, bool hi) {
    return make_uint4(hi ? s.opp[1] : s.own[0], hi ? s.opp[2] : s.own[1], hi ? s.mains : s.own[2],
                      hi ? (uint32_t)s.active : s.opp[0]);
}

__device__ __forceinline__ bool same_state(const uttt_state_t &x, const uttt_state_t &y) {
    return x.own[0] == y.own[0] && x.own[1] == y.own[1] && x.own[2] == y.own[2] && x.opp[0] == y.opp[0] &&
           x.opp[1] == y.opp[1] && x.opp[2] == y.opp[2] && x.mains == y.mains && x.active == y.active;
}

// The table may be shared by several engines whose kernels run concurrently on
// other XCDs, whose L2s are not coherent with this one: every access to flag and
// record is agent-scope (sc1: relaxed agent atomics, or buffer accesses with the
// sc1 bit). Entries are exact (the evaluator is a pure function of the position),
// so any ready entry with a matching key is correct; a reader re-checks the flag
// after copying the values, so an entry rewritten meanwhile is never mixed into the copy.
template <typename T>
__device__ __forceinline__ T ld_agent(const T *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void st_agent(T *p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef float floatx4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
// a wave-uniform slot's record as a 384-byte buffer
__device__ __forceinline__ rsrc_t rec_rsrc(const EvalCache &c, uint32_t slot) {
    slot = (uint32_t)__builtin_amdgcn_readfirstlane((int)slot);
    return __builtin_amdgcn_make_buffer_rsrc(c.rec + (size_t)slot * kRecBytes, 0, kRecBytes, 0x00020000);
}

// Wave-uniform lookup: lanes 0..kProbe-1 read the kProbe slots' flags at once; the first ready slot
// whose tag matches (a hit counts only if no empty slot precedes it in probe order) has its whole
// record read in one round trip (lanes 0-1 the key, checked against s; 2-22 the values), then the
// flag is re-checked. On a hit the 82 values are copied to dst (LDS, 16-byte aligned, >= 84 floats)
// and true is returned; a tag that matched another position's entry (a 16-bit collision) is a miss.
// The probe in two halves: the flags' loads are issued first, so work that does not need them (the select's
// leaf checks) runs under their round trip (round 6)
struct CacheProbe {
    uint64_t h64;
    uint32_t f;  // lane l < kProbe: flag of slot h + l
};
__device__ __forceinline__ CacheProbe cache_probe_issue(const EvalCache &c, const uttt_state_t &s) {
    CacheProbe p;
    p.h64 = 0ull;
    p.f = 0u;
    if (!c.flag) return p;
    const int lane = (int)(threadIdx.x & 63);
    p.h64 = state_hash64(s);
    p.f = lane < kProbe ? ld_agent(c.flag + (((uint32_t)p.h64 + (uint32_t)lane) & c.mask)) : 0u;
    return p;
}

__device__ bool cache_lookup_probed(const EvalCache &c, const CacheProbe &pr, const uttt_state_t &s, float *dst) {
    if (!c.flag) return false;
    const int lane = (int)(threadIdx.x & 63);
    const uint64_t h64 = pr.h64;
    const uint32_t h = (uint32_t)h64, tag = state_tag(h64);
    const uint32_t f = pr.f;
    const uint64_t cand = __ballot(lane < kProbe && flag_ready(f) && flag_tag(f) == tag);
    const uint64_t empty = __ballot(lane < kProbe && f == 0u);
    if (!cand) return false;
    const int hl = __builtin_ctzll(cand);
    if (empty && __builtin_ctzll(empty) < hl) return false;
    const uint32_t hs = (h + (uint32_t)hl) & c.mask;
    const uint32_t f1 = (uint32_t)__builtin_amdgcn_readlane((int)f, hl);
    const rsrc_t r = rec_rsrc(c, hs);
    u32x4_t piece = {0u, 0u, 0u, 0u};
    if (lane < kRecLanes) piece = __builtin_amdgcn_raw_buffer_load_b128(r, 16 * lane, 0, kSc1);
    // seqlock read side: the record loads are served before the re-check is issued; any writer
    // that touched the record since the probe bumped the flag first (claim), so the re-check differs
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint4 kp = key_piece(s, (lane & 1) != 0);
    const bool key_ok = piece[0] == kp.x && piece[1] == kp.y && piece[2] == kp.z && piece[3] == kp.w;
    if (__ballot(lane < 2 && !key_ok)) return false;
    bool ok = true;
    if (lane == 0) ok = ld_agent(c.flag + hs) == f1;
    if (!__shfl(ok, 0)) return false;
    if (lane >= 2 && lane < kRecLanes) *reinterpret_cast<u32x4_t *>(dst + 4 * (lane - 2)) = piece;
    return true;
}

// Wave-level insert of (s -> 81 priors, value): lane l holds prior l in p0 and prior 64 + l in p1
// (l < 17). Lane 0 claims a slot by CAS (flag -> odd); the record is stored as 23 16-byte sc1
// pieces and drained (s_waitcnt vmcnt(0)) before the new flag is published, so a reader on
// any XCD that sees the flag sees the data. A ready slot with this position's tag counts as this
// position (no insert; a 16-bit collision only costs a missed entry), and a concurrent insert of
// the same key may leave a harmless duplicate. When all kProbe slots hold other positions, one of
// them (chosen by the hash) is replaced. Entries are exact, so the table never needs clearing
// while the evaluator is unchanged: it stays warm across moves. Returns whether a record was written.
// sum >= 0 marks `psum` (the sequential f32 sum of the legal priors, uttt_mcts.cpp:150-153, as
// expand_backup computed it) valid: it is stored beside the values (value 82, with 1.0f at 83), so a
// hit expands without re-adding up to 81 priors one dependent add after another.
constexpr int kRecSum = 82, kRecSumFlag = 83;
// A publish held back by cache_insert (defer): the claimed slot and its flag value, stored by the caller once
// its own later stores are drained anyway (k_round1's end of block), so the record's drain is not a round
// trip of its own on the wave's chain (round 6)
struct CachePublish {
    int32_t slot;  // -1: nothing held
    uint32_t pub;
};
__device__ __forceinline__ void cache_publish(const EvalCache &c, const CachePublish &d) {
    if (d.slot < 0 || (threadIdx.x & 63) != 0) return;
    st_agent(c.flag + d.slot, d.pub);
    atomicAdd(stripe_of(c.ctr + 2 * kRow), 1ull);
}

// pr: the kProbe slots' flags for s, loaded ahead (cache_probe_issue, before the expansion's work)
__device__ bool cache_insert(const EvalCache &c, const CacheProbe &pr, const uttt_state_t &s, float p0, float p1, float v,
                             bool has_sum = false, float psum = 0.0f, CachePublish *defer = nullptr) {
    if (!c.flag) return false;
    const int lane = (int)(threadIdx.x & 63);
    int slot = -1;
    uint32_t pub = 0u;
    // the kProbe slots' flags in one round trip (lanes 0..kProbe-1), then lane 0 acts on the first
    // slot that holds this position's tag or is empty; a lost claim falls back to probing one slot
    // after another from there
    const uint64_t h64 = pr.h64;
    const uint32_t h = (uint32_t)h64, tag = state_tag(h64);
    const uint32_t f = pr.f;
    const uint64_t here = __ballot(lane < kProbe && flag_ready(f) && flag_tag(f) == tag);
    const uint64_t free_ = __ballot(lane < kProbe && f == 0u);
    const uint64_t either = here | free_;
    const int first = either ? __builtin_ctzll(either) : kProbe;
    if (lane == 0) {
        bool present = first < kProbe && ((here >> first) & 1ull);
        int i0 = first;
        if (!present && first < kProbe) {
            const uint32_t sl = (h + (uint32_t)first) & c.mask;
            if (atomicCAS(c.flag + sl, 0u, 1u) == 0u) {
                slot = (int)sl;
                pub = flag_publish(0u, tag);
            } else {
                i0 = first + 1;
            }
        }
        for (int i = i0; slot < 0 && !present && i < kProbe; ++i) {
            const uint32_t sl = (h + (uint32_t)i) & c.mask;
            const uint32_t fi = ld_agent(c.flag + sl);
            if (flag_ready(fi) && flag_tag(fi) == tag) {
                present = true;
                break;
            }
            if (fi == 0u && atomicCAS(c.flag + sl, 0u, 1u) == 0u) {
                slot = (int)sl;
                pub = flag_publish(0u, tag);
                break;
            }
        }
        if (slot < 0 && !present) {  // every probe slot taken: replace one (version v -> v + 1 -> v + 2)
            const uint32_t sl = (h + (h >> 29)) & c.mask;
            const uint32_t fr = ld_agent(c.flag + sl);
            if (flag_ready(fr) && atomicCAS(c.flag + sl, fr, fr + 1u) == fr) {
                slot = (int)sl;
                pub = flag_publish(fr, tag);
                atomicAdd(stripe_of(c.ctr + 3 * kRow), 1ull);
            }
        }
    }
    slot = __shfl(slot, 0);
    if (slot < 0) return false;
    pub = (uint32_t)__builtin_amdgcn_readfirstlane((int)pub);
    // piece j of the record: j < 2 the key's words 4j..4j+3, else values 4(j-2)..4(j-2)+3
    // (value e < 64: lane e's p0; e < 81: lane e-64's p1; e == 81: v)
    floatx4_t piece;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int e = 4 * (lane - 2) + i;
        const float a = __shfl(p0, e & 63);
        const float b = __shfl(p1, (e - 64) & 63);
        piece[i] = e < 64 ? a
                          : (e < 81 ? b
                                    : (e == 81 ? v : (e == kRecSum && has_sum ? psum : (e == kRecSumFlag && has_sum ? 1.0f : 0.0f))));
    }
    if (lane < 2) {
        const uint4 kp = key_piece(s, lane != 0);
        piece = floatx4_t{__uint_as_float(kp.x), __uint_as_float(kp.y), __uint_as_float(kp.z), __uint_as_float(kp.w)};
    }
    const rsrc_t r = rec_rsrc(c, (uint32_t)slot);
    // all 24 pieces (the padding as zeros): the record's three 128-byte lines are written whole, so none is
    // a partial-line write at the memory side (round 6; 23 pieces left the third line 112 of 128 bytes)
    if (lane < kRecBytes / 16)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, piece), r, 16 * lane, 0, kSc1);
    if (defer) {  // the caller drains and publishes
        defer->slot = slot;
        defer->pub = pub;
        return true;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    cache_publish(c, CachePublish{slot, pub});
    return true;
}

// ---------------------------------------------------------- expand + backup --
// uttt_mcts.cpp:138-167 for k identical copies of one flushed leaf: priors =
// pol[a] for legal a, sequential f32 sum in action order, divide (uniform
// 1/|legal| if the sum is <= 0); append k child blocks (expand never clears,
// :38-43); back up v k times along path[0..depth] (:47-54, leaf first, sign
// flipping upward). Lane d holds path[d] in path_lo and path[64+d] in path_hi.
// Returns false without writing when the node pool would overflow.
// py (pv_mcts.py:46-56, :104-116): priors normalised by np.sum (float32 pairwise),
// all-zero -> float64 uniform (kMetaP64); ONE child block (expand replaces, and
// the k copies of a flush expand the same children); every node on the path
// gets a network value, so its w becomes float32 (kMetaWF32).
__device__ float np_sum_f32_legal(float p0, float p1, uint64_t b0, uint64_t b1, int L) {
    // numpy pairwise_sum for float32, n <= 128: 8 strided accumulators, then the tail
    auto nth = [&](int idx) -> float {  // idx-th legal prior in action order (wave-uniform)
        const int c0 = __popcll(b0);
        uint64_t bits = idx < c0 ? b0 : b1;
        int r = idx < c0 ? idx : idx - c0;
        for (; r > 0; --r) bits &= bits - 1ull;
        const int l = __builtin_ctzll(bits);
        return idx < c0 ? readlane_f(p0, l) : readlane_f(p1, l);
    };
    if (L < 8) {
        float res = 0.0f;
        for (int i = 0; i < L; ++i) res += nth(i);
        return res;
    }
    float r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = nth(j);
    const int main_end = L - L % 8;
    for (int i = 8; i < main_end; i += 8)
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] += nth(i + j);
    float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (int i = main_end; i < L; ++i) res += nth(i);
    return res;
}

// raw0 / raw1: this lane's prior of action lane / 64 + lane (lane < 17), loaded by the caller
// The sequential f32 sum of the legal priors in action order (uttt_mcts.cpp:150-153): each legal
// prior is stored at its rank in the wave's LDS row (zeros pad the row to a multiple of 4; adding
// +0.0 to a sum that started at +0.0 changes nothing), then every lane reads the row back by
// broadcast 16-byte reads and adds it up in order: one dependent add per prior, instead of a scalar
// find-first-bit, a v_readlane and an add per prior.
__device__ __forceinline__ float seq_sum_legal(float *row /* LDS, 16-B aligned, >= 84 floats */, float p0, float p1,
                                               bool l0, bool l1, int i0, int i1, int L) {
    const int lane = lane_id();
    if (l0) row[i0] = p0;
    if (l1) row[i1] = p1;
    const int L4 = (L + 3) & ~3;
    if (lane >= L && lane < L4) row[lane] = 0.0f;  // L4 - L < 4 <= 64: lanes L .. L4-1 pad
    // the other lanes' stores before any lane's reads (LDS executes a wave's accesses in order; the
    // wait and the clobber keep the compiler from hoisting the reads above the stores)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    float sum = 0.0f;
    const float4 *r4 = reinterpret_cast<const float4 *>(row);
    for (int i = 0; i < L4 / 4; ++i) {
        const float4 q = r4[i];
        sum += q.x;
        sum += q.y;
        sum += q.z;
        sum += q.w;
    }
    return sum;
}

// rec_lo / rec_hi: this lane's path node's record (path[lane] / path[64 + lane]) as the select read it
__device__ bool expand_backup(const Pool &pool, size_t base, int node, int depth, int path_lo, int path_hi,
                              uint4 rec_lo, uint4 rec_hi, int k, const uttt_state_t &s, float raw0, float raw1, float v,
                              int &node_count, bool py = false, float *row = nullptr, bool has_sum = false,
                              float known_sum = 0.0f, float *sum_out = nullptr, uint4 *root_out = nullptr) {
    const int lane = lane_id();
    uint32_t m[3];
    legal_mask(s, m);
    const bool l0 = bit_of(m, lane) != 0u;
    const bool l1 = lane < 17 && bit_of(m, 64 + lane) != 0u;
    const uint64_t b0 = __ballot(l0), b1 = __ballot(l1);
    const int L = __popcll(b0) + __popcll(b1);
    const int nb = node_count;
    const int blocks = py ? 1 : k;
    if ((int64_t)nb + (int64_t)blocks * L > pool.cap || L == 0) return false;
    const int i0 = __popcll(b0 & lanes_below());
    const int i1 = __popcll(b0) + __popcll(b1 & lanes_below());
    const float p0 = l0 ? raw0 : 0.0f;
    const float p1 = l1 ? raw1 : 0.0f;
    float sum = 0.0f;
    if (py) {
        sum = np_sum_f32_legal(p0, p1, b0, b1, L);
    } else if (has_sum) {
        sum = known_sum;  // the cache record's (the same values added in the same order at insert)
    } else if (row) {
        sum = seq_sum_legal(row, p0, p1, l0, l1, i0, i1, L);
    } else {
        for (uint64_t bits = b0; bits; bits &= bits - 1ull) sum += readlane_f(p0, __builtin_ctzll(bits));
        for (uint64_t bits = b1; bits; bits &= bits - 1ull) sum += readlane_f(p1, __builtin_ctzll(bits));
    }
    if (sum_out) *sum_out = sum;
    const float un = 1.0f / (float)L;
    const bool p64 = py && !(sum > 0);  // np.ones(float) / L: float64 priors
    const float q0 = sum > 0 ? p0 / sum : un;
    const float q1 = sum > 0 ? p1 / sum : un;
    const uint4 c0 = new_child(q0, (uint32_t)lane), c1 = new_child(q1, (uint32_t)(64 + lane));
    for (int j = 0; j < blocks; ++j) {
        const size_t blk = base + nb + (size_t)j * L;
        if (l0) pool.rec[blk + i0] = c0;
        if (l1) pool.rec[blk + i1] = c1;
    }
    // the path, leaf (lane depth) to root: w += v k times with the sign flipping upwards, N += k; the
    // leaf also gets its children's block size L and its link (first child, k copies: cpp k blocks,
    // py one block); py: every node on the path now holds a float32 w (kMetaWF32), and the leaf's
    // children carry float64 priors when the policy summed to zero (kMetaP64)
    const uint32_t leaf_meta = (uint32_t)L << 23 | (py ? (kMetaWF32 | (p64 ? kMetaP64 : 0u)) : 0u);
    const uint32_t leaf_link = make_link((uint32_t)nb, (uint32_t)k);
    auto update = [&](uint4 r, int pn, int d) -> uint4 {  // path node pn at depth d, its record r
        float w = __uint_as_float(r.x);
        const float x = ((depth - d) & 1) ? -v : v;
        for (int j = 0; j < k; ++j) w += x;
        r.x = __float_as_uint(w);
        r.z += (uint32_t)k;
        if (py && d < depth) r.z |= kMetaWF32;
        if (d == depth) {
            r.z = (r.z & ~kMetaLMask) | leaf_meta;
            r.w = leaf_link;
        }
        pool.rec[base + pn] = r;
        return r;
    };
    uint4 new_lo = rec_lo;
    if (lane <= depth) new_lo = update(rec_lo, path_lo, lane);
    if (lane + 64 <= depth) update(rec_hi, path_hi, lane + 64);
    if (root_out)  // the root's record as just written (lane 0 holds path[0])
        *root_out = make_uint4((uint32_t)__builtin_amdgcn_readlane((int)new_lo.x, 0),
                               (uint32_t)__builtin_amdgcn_readlane((int)new_lo.y, 0),
                               (uint32_t)__builtin_amdgcn_readlane((int)new_lo.z, 0),
                               (uint32_t)__builtin_amdgcn_readlane((int)new_lo.w, 0));
    node_count = nb + blocks * L;
    return true;
}

// ----------------------------------------------------------- root (begin) --
// uttt_mcts.cpp:92-103: root expanded at once with uniform priors 1.0f/|legal|.
// Self-play passes `live` (slot flags) and the slots' states in place (src_stride = sizeof(Slot)),
// and err: the asynchronous move end's failure word, reset here (once per move, before this move's end,
// after the previous move end's read of it) instead of by a memset on the stream, as is the search's
// failure flag (Trees::count[3]);
// search passes nullptr (all live) and packed states.
__global__ __launch_bounds__(kBlock) void k_begin(Pool pool, Trees tr, const char *src, int src_stride, const int32_t *live,
                                                  unsigned long long *err) {
    const int lane = lane_id();
    const int t = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (t == 0 && lane == 0) {
        if (err) *err = ~0ull;
        tr.count[2] = -1;  // a search starts: no round of it is known to be empty yet (k_round1's fast exit)
        tr.count[3] = 0;   // and no tree of it has failed
    }
    if (t >= tr.n_trees) return;
    const bool on = live ? (live[t] != 0) : true;
    const uttt_state_t s = *reinterpret_cast<const uttt_state_t *>(src + (size_t)t * src_stride);
    const size_t base = (size_t)t * pool.cap;
    uint32_t m[3];
    legal_mask(s, m);
    if (tr.py) {  // pv_mcts.py:134: the root is a plain unexpanded node (evaluated by the first flush)
        const bool any = __ballot(bit_of(m, lane) != 0u) != 0ull || __ballot(lane < 17 && bit_of(m, 64 + lane) != 0u);
        if (lane == 0) {
            pool.rec[base] = make_uint4(0u, 0u, make_meta(kNoAction, 0u), 0u);
            tr.root[t] = s;
            TreeCtl c;
            c.sims_done = 0;
            c.node_count = 1;
            c.status = (on && any) ? kLive : 0;
            c.pad = 0;
            tr.ctl[t] = c;
        }
        return;
    }
    const bool l0 = on && bit_of(m, lane);
    const bool l1 = on && lane < 17 && bit_of(m, 64 + lane);
    const uint64_t b0 = __ballot(l0), b1 = __ballot(l1);
    const int L = __popcll(b0) + __popcll(b1);
    const float up = L ? 1.0f / (float)L : 0.0f;
    if (l0) pool.rec[base + 1 + __popcll(b0 & lanes_below())] = new_child(up, (uint32_t)lane);
    if (l1) pool.rec[base + 1 + __popcll(b0) + __popcll(b1 & lanes_below())] = new_child(up, (uint32_t)(64 + lane));
    if (lane == 0) {
        pool.rec[base] = make_uint4(0u, 0u, make_meta(kNoAction, (uint32_t)L), make_link(L ? 1u : 0u, L ? 1u : 0u));
        tr.root[t] = s;
        TreeCtl c;
        c.sims_done = 0;
        c.node_count = 1 + L;
        c.status = (on && L > 0) ? kLive : 0;
        c.pad = 0;
        tr.ctl[t] = c;
    }
}

// --------------------------------------------------------------- select --
// One wave per tree. uttt_mcts.cpp:109-127 for the simulations up to (and
// including) the next one that reaches an unexpanded non-terminal leaf.
// Terminal simulations are backed up in place (:115-118). The k-1 further
// simulations the reference spends re-finding the same queued leaf are
// accounted by k.
// A launch lasts as long as its slowest tree's chain of dependent loads, and a tree
// whose simulations end on terminals or evaluation-cache hits completes them in place,
// one descent after another. A tree stops after kSelectBudget such completions
// (pending = 2) and resumes in the next launch from the same point: the sequence of
// simulations per tree, hence every result, is unchanged; only the tail of the launch is cut.
constexpr int kSelectBudget = 8;
constexpr int kScanGroup = 4;  // child-scan iterations (64 children each) whose loads are issued together

// k_select phase clock. Product build: empty (every call compiles to nothing). Diagnostics engine
// build (-DUTTT_DIAG_BUILD, libuttt_engine_diag.so, tools/diag/select_cycles.py): each mark drains the
// wave's memory counters, reads s_memtime and charges the cycles since the previous mark to one phase;
// at the end lane 0 adds the wave's phases into g_sel_cyc (all trees, and separately the trees with at
// least kSelHeavyTrips dependent round trips in the launch: the ones that set its length).
enum SelPhase {
    kSpRoot = 0,    // the descent's root link and visits (load wait)
    kSpLoad,        // a child-scan group's loads (wait)
    kSpPuct,        // PUCT values and the per-lane strict '>' scan
    kSpArgmax,      // wave arg-max, winner's registers
    kSpNext,        // next_state, path bookkeeping
    kSpLeaf,        // is_lose / legal count of the leaf
    kSpTerminal,    // terminal backup + fence
    kSpProbe,       // evaluation-cache probe, payload, re-check
    kSpExpand,      // expand + backup of a cache hit (prior sum, child blocks, path)
    kSpHitTail,     // fence + counters after a hit
    kSpQueue,       // pending-leaf record
    kSpRootState,   // the tree's root state (once per launch, before the first descent)
    kSpCount
};
#ifdef UTTT_DIAG_BUILD
constexpr int kSelHeavyTrips = 24;
// per tree (plain read-modify-writes by the tree's own wave: no same-address atomics, which would
// serialize thousands of waves and distort the very latencies measured): [all launches' phases]
// [heavy launches' phases][launches, heavy launches]
constexpr int kSelDiagTrees = 8192;
__device__ unsigned long long g_sel_cyc[kSelDiagTrees][2 * kSpCount + 2];
// the last launch's wall-clock stamps per tree (s_memrealtime, a chip-wide 100 MHz counter): the wave's
// start (its control loads served), its first root phase done, its end; trips in the launch
__device__ unsigned long long g_sel_rt[kSelDiagTrees][4];
// what a live tree's wave loads (and waits for) before its clock starts: 0 nothing, 1 the record 8 past
// its root (another 128-B line of the same page), 2 its root record itself, 3 the record half a pool away
__device__ int g_sel_pretouch;
// the phase sums live in LDS (one row per wave): kept in registers they made k_select spill to
// scratch, whose first accesses are what the diagnostics then measured
__shared__ unsigned long long s_selclk[kWavesPerBlock][kSpCount];
struct SelClock {
    unsigned long long t, rt0, rt1;
    unsigned long long *acc;
    __device__ __forceinline__ void start() {
        acc = s_selclk[threadIdx.x >> 6];
        if ((threadIdx.x & 63) < kSpCount) acc[threadIdx.x & 63] = 0ull;
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        t = __builtin_amdgcn_s_memtime();
        rt0 = __builtin_amdgcn_s_memrealtime();
        rt1 = 0ull;
    }
    template <int P>
    __device__ __forceinline__ void mark() {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        const unsigned long long n = __builtin_amdgcn_s_memtime();
        if (P == kSpRoot && rt1 == 0ull) rt1 = __builtin_amdgcn_s_memrealtime();
        if ((threadIdx.x & 63) == 0) acc[P] += n - t;
        t = n;
    }
    __device__ __forceinline__ void flush(unsigned int trips) {
        const int tree = (int)(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6));
        if ((threadIdx.x & 63) != 0 || tree >= kSelDiagTrees) return;
        g_sel_rt[tree][0] = rt0;
        g_sel_rt[tree][1] = rt1;
        g_sel_rt[tree][2] = __builtin_amdgcn_s_memrealtime();
        g_sel_rt[tree][3] = trips;
        unsigned long long *row = g_sel_cyc[tree];
        const int h = trips >= (unsigned int)kSelHeavyTrips;
#pragma unroll
        for (int i = 0; i < kSpCount; ++i) {
            row[i] += acc[i];
            if (h) row[kSpCount + i] += acc[i];
        }
        row[2 * kSpCount] += 1ull;
        if (h) row[2 * kSpCount + 1] += 1ull;
    }
};
#else
struct SelClock {
    __device__ __forceinline__ void start() {}
    template <int P>
    __device__ __forceinline__ void mark() {}
    __device__ __forceinline__ void flush(unsigned int) {}
};
#endif

// One scan group of NJ x 64 children of a node (uttt_mcts.cpp:62-78). Every load of the group is
// issued before the first compare (one memory round trip per group; a node expanded by a flush of
// k = 8 copies has up to 8 x 81 children), and each child's link word and visits come with it, so
// the winner's are read from its lane's registers after the arg-max instead of from memory. The PUCT
// values of the group are straight-line code: every child's two correctly rounded divisions are
// independent of every other's, so their latencies overlap instead of running one child after
// another behind per-child branches. Children past cnt (clamped loads) never win; the compare is the
// reference's strict '>' in child order.
// pa >= 0: the previous level's winning action, whose next_state runs while this group's loads are in
// flight (it was on the critical path between the arg-max and the next level's loads)
template <int NJ>
__device__ __forceinline__ void puct_group(const uint4 *__restrict__ R, int first, int c0, int cnt, float sq, int lane,
                                           float &best, int &bi, uint4 &bw, uttt_state_t &s, int &pa, SelClock &clk) {
    uint4 r[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) r[j] = R[first + min(c0 + j * kWave + lane, cnt - 1)];
    if (pa >= 0) {
        s = next_state(s, pa);
        pa = -1;
    }
    clk.mark<kSpLoad>();
    float v[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        // uttt_mcts.cpp:70-72, same association and rounding (no FMA: -ffp-contract=off); the
        // reference divides only when n > 0, and an unvisited child's quotient here is discarded
        const int cn = meta_n(r[j].z);
        const float qd = -__uint_as_float(r[j].x) / (float)max(cn, 1);
        const float q = cn > 0 ? qd : 0.0f;
        const float u = __uint_as_float(r[j].y) * sq / (float)(1 + cn);
        v[j] = q + u;
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int c = c0 + j * kWave + lane;
        const bool take = c < cnt && v[j] > best;
        best = take ? v[j] : best;
        bi = take ? c : bi;
        bw.x = take ? r[j].x : bw.x;  // the winner's record: the back-ups start from it, its meta (visits,
        bw.y = take ? r[j].y : bw.y;  // action, L) and link lead the descent on
        bw.z = take ? r[j].z : bw.z;
        bw.w = take ? r[j].w : bw.w;
    }
    clk.mark<kSpPuct>();
}

// The descent of one tree by one wave (k_select's body; k_flush1 runs it after the previous flush's apply).
// cv_row: this wave's 84-float LDS row (a cache hit's values). host_leaf (one-tree searches only): the
// round's counts, the queued leaf and its copies go to fine-grained host memory behind `tag`, and the
// round's device counts / slot 0 are written here (there is no k_scan launch in that form).
// Returns the tree's pending word (wave-uniform), as stored to tr.pending[t].
template <bool PY>
__device__ __forceinline__ int select_wave(Pool pool, Trees tr, EvalCache cache, unsigned long long *stats, int t,
                                           float *cv_row, HostLeaf *host_leaf, int32_t tag, int max_alt = 0,
                                           uttt_state_t *leaf_out = nullptr) {
    // leaf_out (k_round1): a queued leaf's state as stored to tr.leaf[t], so the caller's evaluation reads it
    // from registers (round 6: a store drain and a reload of tr.leaf[t] ended every tree's round)
    const int lane = lane_id();
    TreeCtl ctl = tr.ctl[t];
    // the root's state and record go out with the control word (round 6: they were a second dependent round
    // trip after the status check; a tree with nothing to do discards them)
    const size_t base = (size_t)t * pool.cap;
    uint4 *__restrict__ R = pool.rec + base;
    const uttt_state_t root = tr.root[t];
    const uint4 root_first = R[0];
    int pend = 0;
    unsigned long long bytes = 0;
    unsigned int levels = 0;
    // cache hits / misses of this tree, counted once at the end: an atomic per hit made the next
    // descent's first load wait for it (vmcnt counts the atomic), ~2k cycles a descent (round 4)
    unsigned int hits = 0, misses = 0;
    // dependent round trips of this wave: the control loads (with the root's state and record), then per
    // descent one per child-scan group, and for a completion in place the cache probe, payload and re-check,
    // the path's read-modify-write and the fence
    unsigned int trips = 1;
    SelClock clk;
#ifdef UTTT_DIAG_BUILD
    if (g_sel_pretouch && (ctl.status & kLive)) {
        const uint4 *pr = pool.rec + (size_t)t * pool.cap;
        const int off = g_sel_pretouch == 1 ? 8 : (g_sel_pretouch == 2 ? 0 : (int)(pool.cap / 2));
        const uint32_t q = pr[off].x;
        asm volatile("s_waitcnt vmcnt(0)" ::"v"(q) : "memory");
    }
#endif
    clk.start();
    if ((ctl.status & kLive) && !(ctl.status & kErrMask) && ctl.sims_done < tr.sims) {
        clk.mark<kSpRootState>();
        int sims_done = ctl.sims_done;
        int budget = tr.budget;
        // the root's record: as loaded with the control word, then after this wave's own last back-up (no
        // other wave writes this tree's nodes during the launch): no descent reloads R[0]
        uint4 root_rec = root_first;
        for (;;) {
            uttt_state_t s = root;
            int node = 0, depth = 0;
            int path_lo = 0, path_hi = 0;  // lane d: path[d], path[64 + d]
            // the current node's meta (visits, action, L) and link (below the root: from the parent's scan)
            const uint4 r0 = root_rec;
            uint2 nm = make_uint2(r0.z, r0.w);
            // lane d: the record of path[d] (prec_lo) and path[64 + d] (prec_hi) as read on the way down
            uint4 prec_lo = r0, prec_hi = make_uint4(0u, 0u, 0u, 0u);
            clk.mark<kSpRoot>();
            bool fail = false;
            int pa = -1;  // a winning action whose next_state is pending (applied under the next loads)
            for (;;) {
                const int cnt = PY ? meta_L(nm.x) : link_k(nm.y) * meta_L(nm.x);
                if (cnt == 0) break;
                const int first = link_first(nm.y);
                const int kself = (node == 0 && !PY) ? 0 : link_k(nm.y);
                const int total = meta_n(nm.x) - kself;  // == sum of children's visits
                int bi = kNone;
                uint4 wr = make_uint4(0u, 0u, 0u, 0u);  // the chosen child's record
                if (!PY) {
                    const float sq = sqrtf((float)total);
                    float best = -1e9f;
                    uint4 bw = make_uint4(0u, 0u, 0u, 0u);
                    // Every load of a group of kScanGroup x 64 children is issued before the first
                    // compare (one memory round trip per group; a node expanded by a flush of k = 8
                    // copies has up to 8 x 81 children), and each child's link word and visits come
                    // with it, so the winner's are read from its lane's registers instead of from
                    // memory after the arg-max: one dependent round trip per level.
                    for (int c0 = 0; c0 < cnt; c0 += kScanGroup * kWave) {
                        ++trips;
                        if (cnt - c0 <= kWave) puct_group<1>(R, first, c0, cnt, sq, lane, best, bi, bw, s, pa, clk);
                        else puct_group<kScanGroup>(R, first, c0, cnt, sq, lane, best, bi, bw, s, pa, clk);
                    }
                    bi = wave_argmax(best, bi, cnt);
                    if (bi != kNone) {  // the winner's lane holds its record
                        const int wl = bi & (kWave - 1);
                        wr = make_uint4((uint32_t)__builtin_amdgcn_readlane((int)bw.x, wl),
                                        (uint32_t)__builtin_amdgcn_readlane((int)bw.y, wl),
                                        (uint32_t)__builtin_amdgcn_readlane((int)bw.z, wl),
                                        (uint32_t)__builtin_amdgcn_readlane((int)bw.w, wl));
                        nm = make_uint2(wr.z, wr.w);
                    }
                    clk.mark<kSpArgmax>();
                } else {
                    trips += 2u + (unsigned int)((cnt + kWave - 1) / kWave);  // the node's record, the scan
                    // pv_mcts.py:120-130 under NumPy 2 promotion: float32 ops with sqrt(t)
                    // in double, or float64 throughout when the priors are float64;
                    // np.argmax: first maximum, a NaN counts as the maximum. (k_apply refuses a
                    // non-finite legal prior or value in both semantics, UTTT_ERR_NONFINITE, where
                    // pv_mcts.py would keep searching, so no NaN statistic reaches this scan today;
                    // the branch keeps the scan a complete restatement of np.argmax)
                    const bool p64 = (nm.x & kMetaP64) != 0u;
                    const double sqt = sqrt((double)total);
                    const float sq = (float)sqt;
                    const double pu = 1.0 / (double)meta_L(nm.x);
                    double best = -HUGE_VAL;
                    for (int c = lane; c < cnt; c += kWave) {
                        const uint4 rc = R[first + c];
                        const int cn = meta_n(rc.z);
                        const float cw = __uint_as_float(rc.x);
                        const bool wf = (rc.z & kMetaWF32) != 0u;
                        double v;
                        if (p64) {
                            const double q = cn > 0 ? (wf ? (double)((-cw) / (float)cn) : (double)(-cw) / (double)cn) : 0.0;
                            v = q + ((1.0 * pu) * sqt) / (double)(1 + cn);
                        } else {
                            const float q = cn > 0 ? (wf ? (-cw) / (float)cn : (float)((double)(-cw) / (double)cn)) : 0.0f;
                            const float u = ((1.0f * __uint_as_float(rc.y)) * sq) / (float)(1 + cn);
                            v = (double)(q + u);
                        }
                        if (v != v) v = HUGE_VAL;
                        if (bi == kNone || v > best) {
                            best = v;
                            bi = c;
                        }
                    }
                    wave_argmax_d(best, bi);
                }
                bi = __builtin_amdgcn_readfirstlane(bi);
                bytes += 12ull * (unsigned long long)cnt + 8ull;
                if (bi == kNone) {  // every child NaN: the reference would dereference null
                    fail = true;
                    if (lane == 0) {
                        ctl.status |= kErrSelect;
                        flag_tree_error(tr);
                    }
                    break;
                }
                node = first + bi;
                ++depth;
                if (depth >= kMaxDepth) {
                    fail = true;
                    if (lane == 0) {
                        ctl.status |= kErrDepth;
                        flag_tree_error(tr);
                    }
                    break;
                }
                if (PY) {
                    wr = R[node];
                    nm = make_uint2(wr.z, wr.w);
                }
                if (lane == (depth & 63)) {
                    if (depth < 64) {
                        path_lo = node;
                        prec_lo = wr;
                    } else {
                        path_hi = node;
                        prec_hi = wr;
                    }
                }
                if (PY) s = next_state(s, meta_action(nm.x));
                else pa = meta_action(nm.x);
                clk.mark<kSpNext>();
            }
            if (pa >= 0) s = next_state(s, pa);  // the leaf's state
            if (fail) break;
            levels += (unsigned int)(depth + 1);
            // the evaluation cache's flags for this leaf are loaded before its terminal checks, which run
            // under that round trip (a terminal leaf's probe is discarded)
            const CacheProbe probe = cache_probe_issue(cache, s);
            const bool lose = is_lose(s);
            const bool no_legal = legal_count(s) == 0u;
            clk.mark<kSpLeaf>();
            if (lose || no_legal) {
                // Terminal: search_leaf returns -(is_lose ? -1 : 0) (uttt_mcts.cpp:19-22),
                // backpropagate adds it at the leaf and flips sign upwards (:47-54).
                const float v = -(lose ? -1.0f : 0.0f);
                auto backup1 = [&](uint4 r, int pn, int d) -> uint4 {  // from the record read on the way down
                    r.x = __float_as_uint(__uint_as_float(r.x) + (((depth - d) & 1) ? -v : v));
                    r.z += 1u;
                    R[pn] = r;
                    return r;
                };
                uint4 nl = prec_lo;
                if (lane <= depth) nl = backup1(prec_lo, path_lo, lane);
                if (lane + 64 <= depth) backup1(prec_hi, path_hi, lane + 64);
                root_rec = make_uint4((uint32_t)__builtin_amdgcn_readlane((int)nl.x, 0),
                                      (uint32_t)__builtin_amdgcn_readlane((int)nl.y, 0),
                                      (uint32_t)__builtin_amdgcn_readlane((int)nl.z, 0),
                                      (uint32_t)__builtin_amdgcn_readlane((int)nl.w, 0));
                wave_memory_fence();
                trips += 2;
                bytes += 16ull * (unsigned long long)(depth + 1);
                clk.mark<kSpTerminal>();
                ++sims_done;
                if (sims_done >= tr.sims) break;
                if (--budget == 0) {
                    pend = 2;
                    break;
                }
                continue;
            }
            // Unexpanded leaf (n == 0 && no children, uttt_mcts.cpp:121): queue it with
            // k = the copies the reference would queue before flushing (:127).
            const int k = min(tr.batch, tr.sims - sims_done);
            float *cv = cv_row;
            trips += cache.flag ? 1 : 0;
            const bool hit = cache_lookup_probed(cache, probe, s, cv);
            clk.mark<kSpProbe>();
            if (hit) {  // the flush's evaluation is already known: apply it now
                trips += 4;
                // cv doubles as the prior sum's row: its values are in registers before the call
                const float h0 = cv[lane], h1 = lane < 17 ? cv[64 + lane] : 0.0f, hv = cv[81];
                const bool hs = !PY && cv[kRecSumFlag] == 1.0f;
                if (!expand_backup(pool, base, node, depth, path_lo, path_hi, prec_lo, prec_hi, k, s, h0, h1, hv,
                                   ctl.node_count, PY, cv, hs, cv[kRecSum], nullptr, &root_rec)) {
                    if (lane == 0) {
                        ctl.status |= kErrCapacity;
                        flag_tree_error(tr);
                    }
                    break;
                }
                clk.mark<kSpExpand>();
                wave_memory_fence();
                ++hits;
                // the probe's flags, the record, the k child blocks and the path's records
                bytes += 32ull + 368ull + 16ull * (unsigned long long)(k * (int)legal_count(s)) + 16ull * (depth + 1);
                clk.mark<kSpHitTail>();
                sims_done += k;
                if (sims_done >= tr.sims) break;
                if (--budget == 0) {
                    pend = 2;
                    break;
                }
                continue;
            }
            misses += cache.flag ? 1u : 0u;
            int32_t *gp = tr.path + (size_t)t * kMaxDepth;
            uint4 *gr = tr.path_rec + (size_t)t * kMaxDepth;
            if (lane <= depth) {
                gp[lane] = path_lo;
                gr[lane] = prec_lo;
            }
            if (lane + 64 <= depth) {
                gp[lane + 64] = path_hi;
                gr[lane + 64] = prec_hi;
            }
            if (lane == 0) {
                LeafRec r;
                r.node = node;
                r.depth = depth;
                r.k = k;
                r.pad = 0;
                tr.rec[t] = r;
                tr.leaf[t] = s;
            }
            if (leaf_out) *leaf_out = s;
            // the probe's flags, the queued path (indices and records), LeafRec and state
            bytes += (cache.flag ? 32ull : 0ull) + 20ull * (unsigned long long)(depth + 1) + 48ull;
            // 3: this leaf's k simulations leave the tree more to do (after its apply)
            pend = (sims_done + k < tr.sims ? 3 : 1) | depth << 8;
            clk.mark<kSpQueue>();
            break;
        }
        ctl.sims_done = sims_done;
        if (lane == 0) tr.ctl[t] = ctl;
    }
    clk.flush(trips);
    if (lane == 0) {
        tr.pending[t] = pend;
        if (hits) atomicAdd(stripe_of(cache.ctr), (unsigned long long)hits);
        if (misses) atomicAdd(stripe_of(cache.ctr + kRow), (unsigned long long)misses);
        if (stats && bytes) atomicAdd(stripe_of(stats + kKSelect * kRow), bytes);
        if (stats && levels) {
            atomicAdd(stripe_of(stats + kKSelLevels * kRow), (unsigned long long)levels);
            atomicAdd(stripe_of(stats + kKSelTrees * kRow), 1ull);
            atomicMax(stripe_of(stats + (max_alt ? kKSelMaxB : kKSelMax) * kRow), (unsigned long long)levels);
            atomicAdd(stripe_of(stats + kKSelTrips * kRow), (unsigned long long)trips);
            atomicMax(stripe_of(stats + (max_alt ? kKSelTripMaxB : kKSelTripMax) * kRow), (unsigned long long)trips);
        }
        if (host_leaf) {  // one tree: what k_scan would derive from pending[0]
            const int p = pend & 0xFF, c0 = (p == 1 || p == 3) ? 1 : 0, c1 = p == 2 ? 1 : 0, c2 = p >= 2 ? 1 : 0;
            tr.count[0] = c0;
            tr.count[1] = c1;
            tr.count[2] = c2;
            tr.tree_of[0] = t;
            tr.depth_of[0] = pend >> 8;
            __hip_atomic_store(&host_leaf->count, c0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&host_leaf->stopped, c1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&host_leaf->left, c2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (c0) {
                const uttt_state_t st = tr.leaf[t];  // stored by this lane above
                const int32_t *w = reinterpret_cast<const int32_t *>(&st);
                int32_t *d = reinterpret_cast<int32_t *>(&host_leaf->state);
#pragma unroll
                for (int i = 0; i < 8; ++i) __hip_atomic_store(d + i, w[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(&host_leaf->k, tr.rec[t].k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            host_stores_done();
            st_host(&host_leaf->tag, tag);
        }
    }
    return __builtin_amdgcn_readfirstlane(pend);
}

template <bool PY>
__global__ __launch_bounds__(kBlock, 4) void k_select(Pool pool, Trees tr, EvalCache cache,
                                                   unsigned long long *stats) {
    __shared__ __attribute__((aligned(16))) float s_hit[kWavesPerBlock][84];  // a cache hit's values, per wave
    const int t = wave_index();
    if (t >= tr.n_trees) return;
    select_wave<PY>(pool, tr, cache, stats, t, s_hit[threadIdx.x >> 6], nullptr, 0);
}

// ------------------------------------------------------------------- scan --
// Exclusive prefix sum of one value per thread over a 1,024-thread block (16 waves): a wave scan
// by lane shifts, the 16 wave totals scanned by the first wave through LDS; two barriers where
// a Hillis-Steele scan over LDS takes twenty. Returns the exclusive prefix; *total gets the sum.
template <typename T>
__device__ __forceinline__ T block_scan_1024(T v, T *total, T *wsum /* __shared__ [16] */) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    T x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const T t = __shfl_up(x, off);
        if (lane >= off) x += t;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    if (wave == 0) {
        T w = lane < 16 ? wsum[lane] : T(0);
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
            const T t = __shfl_up(w, off);
            if (lane >= off) w += t;
        }
        if (lane < 16) wsum[lane] = w;
    }
    __syncthreads();
    *total = wsum[15];
    return x - v + (wave > 0 ? wsum[wave - 1] : T(0));
}

// Two exclusive scans over the block in one pass (the barriers and the wave-0 step shared): k_finalize's
// finished lengths and its packed (free, finished) counts (round 6: two passes of block_scan_1024 before)
__device__ __forceinline__ void block_scan2_1024(unsigned long long &a, unsigned long long &c,
                                                 unsigned long long *a_tot, unsigned long long *c_tot,
                                                 unsigned long long *wsum /* __shared__ [32] */) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    unsigned long long x = a, y = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const unsigned long long tx = __shfl_up(x, off), ty = __shfl_up(y, off);
        if (lane >= off) {
            x += tx;
            y += ty;
        }
    }
    if (lane == 63) {
        wsum[wave] = x;
        wsum[16 + wave] = y;
    }
    __syncthreads();
    if (wave == 0) {
        unsigned long long w = lane < 32 ? wsum[lane] : 0ull;  // lanes 0-15: a's wave sums, 16-31: c's
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
            const unsigned long long t = __shfl_up(w, off);
            if ((lane & 15) >= off) w += t;
        }
        if (lane < 32) wsum[lane] = w;
    }
    __syncthreads();
    *a_tot = wsum[15];
    *c_tot = wsum[31];
    a = x - a + (wave > 0 ? wsum[wave - 1] : 0ull);
    c = y - c + (wave > 0 ? wsum[16 + wave - 1] : 0ull);
}

// One block: exclusive scan of pending flags -> tree_of[slot] in tree order.
// host_count (optional): the three counts are also stored to this host-visible (fine-grained pinned)
// word triple at system scope, so the host reads a round's counts when the round's event completes
// without a copy operation on the stream (round 4: one stream operation less per round). Round 5: word 3
// gets the round's tag after them (a system-scope release store), so a host that polls the tag needs no
// event either (uttt_round_hash_async).
__global__ __launch_bounds__(1024) void k_scan(Trees tr, unsigned long long *stats, int32_t *host_count, int32_t tag) {
    __shared__ unsigned long long wsum[16];
    const int tid = threadIdx.x;
    if (stats && tid < 64) {  // the select launch before this scan is complete: fold its slowest tree
        // (the max over the stripes, one per lane of the first wave)
        unsigned long long ml = 0ull, mt = 0ull;
        if (tid < kStripes) {
            unsigned long long *a = stats + kKSelMax * kRow + tid * kStripeStride;
            unsigned long long *b = stats + kKSelTripMax * kRow + tid * kStripeStride;
            ml = *a;
            mt = *b;
            *a = 0ull;
            *b = 0ull;
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const unsigned long long ol = __shfl_xor(ml, off), ot = __shfl_xor(mt, off);
            ml = ol > ml ? ol : ml;
            mt = ot > mt ? ot : mt;
        }
        if (tid == 0) {
            stats[kKSelMaxSum * kRow] += ml;
            stats[kKSelTripMaxSum * kRow] += mt;
        }
    }
    const int per = (tr.n_trees + 1023) / 1024;
    const int b = tid * per, e = min(b + per, tr.n_trees);
    // up to kScanPer flags per thread (4,096 trees) are loaded together and kept for the second pass (round 5:
    // the two loops each waited for one load per tree in turn); more per thread are re-read there
    constexpr int kScanPer = 4;
    int held[kScanPer];
#pragma unroll
    for (int j = 0; j < kScanPer; ++j) held[j] = b + j < e ? tr.pending[b + j] : 0;
    unsigned long long local = 0, cap = 0, mo = 0;
    for (int i = b; i < e; ++i) {
        const int p = (i - b < kScanPer ? held[i - b] : tr.pending[i]) & 0xFF;
        local += p == 1 || p == 3;
        cap += p == 2;
        mo += p >= 2;
    }
    // the three counts in 21-bit fields of one scanned word (each total <= n_trees < 2^21)
    unsigned long long tot;
    const unsigned long long ex = block_scan_1024(local | (cap << 21) | (mo << 42), &tot, wsum);
    int slot = (int)(ex & 0x1FFFFFull);
    for (int i = b; i < e; ++i) {
        const int p = i - b < kScanPer ? held[i - b] : tr.pending[i];
        if ((p & 1) != 0) {  // 1 or 3
            tr.depth_of[slot] = p >> 8;
            tr.slot_of[i] = slot;
            tr.tree_of[slot++] = i;
        } else {
            tr.slot_of[i] = -1;
        }
    }
    if (tid == 0) {
        const int c0 = (int)(tot & 0x1FFFFFull), c1 = (int)((tot >> 21) & 0x1FFFFFull);
        const int c2 = (int)(tot >> 42);  // trees with simulations left after this round (0: the search ends with it)
        tr.count[0] = c0;
        tr.count[1] = c1;
        tr.count[2] = c2;
        if (host_count) {
            __hip_atomic_store(host_count + 0, c0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(host_count + 1, c1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(host_count + 2, c2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            host_stores_done();
            st_host(host_count + 3, tag);
        }
    }
}

// ----------------------------------------------------------------- encode --
// The network input of each pending leaf (uttt_game.cpp:244-280 transposed to
// NCHW as pv_mcts_cpp.py:57-60 does): ch0 own stones, ch1 opponent, ch2 legal.
__global__ __launch_bounds__(256) void k_encode(Trees tr, float *__restrict__ x, int n) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n * 243) return;
    const int slot = g / 243, j = g % 243;
    const int ch = j / 81, pos = j % 81;
    const uttt_state_t s = tr.leaf[tr.tree_of[slot]];
    const int a = action_at(pos);
    uint32_t bit;
    if (ch == 0) bit = bit_of(s.own, a);
    else if (ch == 1) bit = bit_of(s.opp, a);
    else {
        uint32_t m[3];
        legal_mask(s, m);
        bit = bit_of(m, a);
    }
    x[g] = bit ? 1.0f : 0.0f;
}

// ------------------------------------------------------------------ apply --
// One wave per pending leaf (uttt_mcts.cpp:138-167 for each of its k copies):
// legal priors, sequential f32 sum in action order, divide (uniform 1/|legal|
// if sum <= 0), append the child block, back up the value along the path.
// per_copy: row rowbase[slot] + j holds copy j's result; else row = slot.
__device__ __forceinline__ void apply_wave(Pool pool, Trees tr, EvalCache cache, const float *__restrict__ policy,
                                           int64_t pld, const float *__restrict__ value, int64_t vld,
                                           const int32_t *__restrict__ rowbase, int per_copy,
                                           unsigned long long *bytes_ctr, int slot, float *row /* LDS, 84 floats */,
                                           int by_tree = -1, int by_tree_depth = 0, float *copy_rows = nullptr,
                                           bool host_rows = false, CachePublish *defer = nullptr) {
    // copy_rows (LDS, 8 x 84 floats, 16-B aligned; optional): the per-copy prior sums of a chunk run in 8 lanes
    // at once instead of one copy after another. host_rows: the evaluation rows sit in fine-grained host
    // memory the host wrote behind a polled command; they are read with system-coherent (sc0 sc1) loads,
    // so no cache invalidation stands between the command and them (k_search1: one leaf, its rows from row 0,
    // at least 8 rows readable)
    auto ld_row = [host_rows](const float *a) -> float {
        return host_rows ? __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : *a;
    };
    const int lane = lane_id();
    // two dependent round trips before the work: the count with this slot's tree and leaf depth
    // (tree_of / depth_of hold n_trees entries, stale past the count), then the tree's records, the
    // path entries 0..depth (round 4: all 128 were loaded, 2.5 KB a leaf) and the slot's evaluation.
    // by_tree >= 0 (one-dispatch hash rounds, k_round1): the tree and its leaf's depth are given and its
    // evaluation is row `slot` == by_tree (rows by tree, no scan)
    int t, dq;
    if (by_tree >= 0) {
        t = by_tree;
        dq = by_tree_depth;
    } else {
        const int cnt = tr.count[0];
        t = tr.tree_of[slot < tr.n_trees ? slot : 0];
        dq = tr.depth_of[slot < tr.n_trees ? slot : 0];
        if (slot >= cnt) return;
    }
    // host_rows, per copy: the first 8 rows (the host block holds at least 16) are loaded before the tree's
    // records, whose round trip they then share; masked by legality and by k once those have arrived
    constexpr int kCopyChunk = 8;
    float h0[kCopyChunk], h1[kCopyChunk], hv[kCopyChunk];
    if (host_rows && per_copy) {
#pragma unroll
        for (int jj = 0; jj < kCopyChunk; ++jj) {
            const float *pol = policy + (int64_t)jj * pld;
            h0[jj] = ld_row(pol + lane);
            h1[jj] = ld_row(pol + 64 + (lane < 17 ? lane : 16));
            hv[jj] = ld_row(value + (int64_t)jj * vld);
        }
    }
    const LeafRec r = tr.rec[t];
    TreeCtl ctl = tr.ctl[t];
    const uttt_state_t s = tr.leaf[t];
    const size_t base = (size_t)t * pool.cap;
    const int32_t *gp = tr.path + (size_t)t * kMaxDepth;
    const uint4 *gr = tr.path_rec + (size_t)t * kMaxDepth;
    int g_lo = 0, g_hi = 0;
    uint4 pr_lo = {0u, 0u, 0u, 0u}, pr_hi = {0u, 0u, 0u, 0u};  // the path nodes' records as the select read them
    if (lane <= dq) {
        g_lo = gp[lane];
        pr_lo = gr[lane];
    }
    if (lane + 64 <= dq) {
        g_hi = gp[lane + 64];
        pr_hi = gr[lane + 64];
    }
    float raw0 = 0.0f, raw1 = 0.0f, rawv = 0.0f;
    if (!per_copy) {
        const float *pol = policy + (int64_t)slot * pld;
        raw0 = ld_row(pol + lane);
        raw1 = ld_row(pol + 64 + (lane < 17 ? lane : 16));
        rawv = ld_row(value + (int64_t)slot * vld);
    }
    const int depth = r.depth;
    const int k = r.k;
    const int pn_lo = lane <= depth ? g_lo : 0;
    const int pn_hi = lane + 64 <= depth ? g_hi : 0;
    int L = 0;
    bool inserted = false;
    const int nodes_before = ctl.node_count;
    if (!per_copy) {
        const float v = rawv;
        // SURVEY §5 failure detection: a NaN / Inf legal prior or value (uttt_mcts.cpp:144-166 would
        // expand and back it up silently) stops the tree with kErrNonFinite, which the host raises at
        // the move boundary (UTTT_ERR_NONFINITE); nothing of it is expanded or cached. A non-finite
        // entry of an illegal action is never read by the search (it is expanded as the reference
        // would), but such a row is not cached either: the table only ever holds finite rows.
        const bool fin0 = __builtin_isfinite(raw0), fin1 = __builtin_isfinite(raw1);
        {
            uint32_t m[3];
            legal_mask(s, m);
            const bool bad = (bit_of(m, lane) && !fin0) || (lane < 17 && bit_of(m, 64 + lane) && !fin1) ||
                             !__builtin_isfinite(v);
            if (__ballot(bad)) {
                if (lane == 0) {
                    ctl.status |= kErrNonFinite;
                    tr.ctl[t] = ctl;
                    flag_tree_error(tr);
                }
                return;
            }
        }
        const bool cacheable = __ballot(!fin0 || (lane < 17 && !fin1)) == 0ull;
        // the insert's flag loads go out before the expansion's work, which runs under their round trip
        const CacheProbe ipr = cache_probe_issue(cache, s);
        float psum = 0.0f;
        if (!expand_backup(pool, base, r.node, depth, pn_lo, pn_hi, pr_lo, pr_hi, k, s, raw0, lane < 17 ? raw1 : 0.0f,
                           v, ctl.node_count, tr.py != 0, row, false, 0.0f, &psum)) {
            if (lane == 0) {
                ctl.status |= kErrCapacity;
                tr.ctl[t] = ctl;
                flag_tree_error(tr);
            }
            return;
        }
        inserted = cacheable && cache_insert(cache, ipr, s, raw0, raw1, v, tr.py == 0, psum, defer);
        L = (ctl.node_count - nodes_before) / k;
    } else {
        // the reference's exact call pattern: k results, one per queued copy, applied in order
        uint32_t m[3];
        legal_mask(s, m);
        const bool l0 = bit_of(m, lane) != 0u;
        const bool l1 = lane < 17 && bit_of(m, 64 + lane) != 0u;
        const uint64_t b0 = __ballot(l0), b1 = __ballot(l1);
        L = __popcll(b0) + __popcll(b1);
        const int i0 = __popcll(b0 & lanes_below());
        const int i1 = __popcll(b0) + __popcll(b1 & lanes_below());
        const int nb = ctl.node_count;
        if ((int64_t)nb + (int64_t)k * L > pool.cap || L == 0) {
            if (lane == 0) {
                ctl.status |= kErrCapacity;
                tr.ctl[t] = ctl;
                flag_tree_error(tr);
            }
            return;
        }
        // the copies' rows in chunks of kCopyChunk whose loads are all issued before the first use: one
        // memory round trip per chunk instead of one per copy (the rows of a one-tree search sit in host
        // memory, a PCIe round trip each: round 6 measured 16 us of a flush's apply on 8 sequential rows)
        const int64_t rb = rowbase[slot];
        float c0[kCopyChunk], c1[kCopyChunk], cv[kCopyChunk];
        auto load_chunk = [&](int j0) {
            if (host_rows && j0 == 0) {  // the prefetched rows (row base 0)
#pragma unroll
                for (int jj = 0; jj < kCopyChunk; ++jj) {
                    const int q = jj < k ? jj : 0;
                    float x0 = h0[0], x1 = h1[0], xv = hv[0];
#pragma unroll
                    for (int i = 1; i < kCopyChunk; ++i) {
                        x0 = q == i ? h0[i] : x0;
                        x1 = q == i ? h1[i] : x1;
                        xv = q == i ? hv[i] : xv;
                    }
                    c0[jj] = l0 ? x0 : 0.0f;
                    c1[jj] = l1 ? x1 : 0.0f;
                    cv[jj] = xv;
                }
                return;
            }
#pragma unroll
            for (int jj = 0; jj < kCopyChunk; ++jj) {
                const int64_t row = rb + (j0 + jj < k ? j0 + jj : j0);
                const float *pol = policy + row * pld;
                c0[jj] = l0 ? ld_row(pol + lane) : 0.0f;
                c1[jj] = l1 ? ld_row(pol + 64 + lane) : 0.0f;
                cv[jj] = ld_row(value + row * vld);
            }
        };
        // copy_rows: lane jj's sum of the chunk's copy jj, its legal priors compacted in action order into an
        // LDS row (seq_sum_legal's order and zero padding, so the same f32 sum as the one-lane loop below)
        const int L4 = (L + 3) & ~3;
        float csum = 0.0f;
        auto chunk_sums = [&]() {
#pragma unroll
            for (int jj = 0; jj < kCopyChunk; ++jj) {
                float *rw = copy_rows + jj * 84;
                if (l0) rw[i0] = c0[jj];
                if (l1) rw[i1] = c1[jj];
                if (lane >= L && lane < L4) rw[lane] = 0.0f;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every lane's stores before any lane's reads
            const float4 *r4 = reinterpret_cast<const float4 *>(copy_rows + (lane & (kCopyChunk - 1)) * 84);
            float acc = 0.0f;
            for (int i = 0; i < L4 / 4; ++i) {
                const float4 q = r4[i];
                acc += q.x;
                acc += q.y;
                acc += q.z;
                acc += q.w;
            }
            csum = acc;
        };
        bool bad = false;  // any copy's legal prior or value non-finite: nothing is applied (as above)
        for (int j0 = 0; j0 < k; j0 += kCopyChunk) {
            load_chunk(j0);
#pragma unroll
            for (int jj = 0; jj < kCopyChunk; ++jj)
                bad |= !__builtin_isfinite(c0[jj]) || !__builtin_isfinite(c1[jj]) || !__builtin_isfinite(cv[jj]);
        }
        if (__ballot(bad)) {
            if (lane == 0) {
                ctl.status |= kErrNonFinite;
                tr.ctl[t] = ctl;
                flag_tree_error(tr);
            }
            return;
        }
        uint4 r_lo = pr_lo, r_hi = pr_hi;
        float w_lo = __uint_as_float(r_lo.x), w_hi = __uint_as_float(r_hi.x);
        for (int j = 0; j < k; ++j) {
            const int jj = j & (kCopyChunk - 1);
            if (jj == 0 && k > kCopyChunk) load_chunk(j);  // k <= kCopyChunk: the check's chunk is still held
            if (jj == 0 && copy_rows) chunk_sums();
            float p0 = c0[0], p1 = c1[0], v = cv[0];
#pragma unroll
            for (int i = 1; i < kCopyChunk; ++i) {
                p0 = jj == i ? c0[i] : p0;
                p1 = jj == i ? c1[i] : p1;
                v = jj == i ? cv[i] : v;
            }
            float sum = 0.0f;
            if (copy_rows) {
                sum = readlane_f(csum, jj);
            } else {
                for (uint64_t bits = b0; bits; bits &= bits - 1ull) sum += readlane_f(p0, __builtin_ctzll(bits));
                for (uint64_t bits = b1; bits; bits &= bits - 1ull) sum += readlane_f(p1, __builtin_ctzll(bits));
            }
            const float un = 1.0f / (float)L;
            const float q0 = sum > 0 ? p0 / sum : un;
            const float q1 = sum > 0 ? p1 / sum : un;
            const size_t blk = base + nb + (size_t)j * L;
            if (l0) pool.rec[blk + i0] = new_child(q0, (uint32_t)lane);
            if (l1) pool.rec[blk + i1] = new_child(q1, (uint32_t)(64 + lane));
            if (lane <= depth) w_lo += ((depth - lane) & 1) ? -v : v;
            if (lane + 64 <= depth) w_hi += ((depth - lane - 64) & 1) ? -v : v;
        }
        // path nodes: w, N += k; the leaf (depth) also gets L and its link (first child, k blocks)
        auto put = [&](uint4 rr, float w, int pn, int d) {
            rr.x = __float_as_uint(w);
            rr.z += (uint32_t)k;
            if (d == depth) {
                rr.z = (rr.z & ~kMetaLMask) | ((uint32_t)L << 23);
                rr.w = make_link((uint32_t)nb, (uint32_t)k);
            }
            pool.rec[base + pn] = rr;
        };
        if (lane <= depth) put(r_lo, w_lo, pn_lo, lane);
        if (lane + 64 <= depth) put(r_hi, w_hi, pn_hi, lane + 64);
        ctl.node_count = nb + k * L;
    }
    if (lane == 0) {
        ctl.sims_done += k;
        tr.ctl[t] = ctl;
        if (bytes_ctr) {
            // algorithmic bytes of one leaf: the slot's tree, depth and count (12), its LeafRec, TreeCtl and
            // state (64), the path's indices and records (20 per level), the evaluation (328 per copy);
            // written: the k child blocks (16 per child), the path's records (16 per level), the TreeCtl
            // (16); with the evaluation cache: the probe's 8 flags (32) and a new record (368 + 4)
            const int copies = per_copy ? k : 1;
            const unsigned long long b = 12ull + 64ull + 36ull * (unsigned long long)(depth + 1) + 328ull * copies +
                                         16ull * (unsigned long long)(k * L) + 16ull + (cache.flag ? 32ull : 0ull) +
                                         (inserted ? 372ull : 0ull);
            atomicAdd(stripe_of(bytes_ctr), b);
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_apply(Pool pool, Trees tr, EvalCache cache, const float *__restrict__ policy,
                                                  int64_t pld, const float *__restrict__ value, int64_t vld,
                                                  const int32_t *__restrict__ rowbase, int per_copy,
                                                  unsigned long long *bytes_ctr) {
    __shared__ __attribute__((aligned(16))) float s_row[kWavesPerBlock][84];  // the prior sum's row, per wave
    apply_wave(pool, tr, cache, policy, pld, value, vld, rowbase, per_copy, bytes_ctr, wave_index(),
               s_row[threadIdx.x >> 6]);
}

// One flush of a one-tree search in one launch (round 5, uttt_search_select_host / _apply_host): the previous
// flush's evaluation applied (k_apply's body, reading it from pinned host memory), then the next descent
// (k_select's body), which stores the round's result to pinned host memory behind its tag. One wave, one
// dispatch per flush where k_apply, k_select and k_scan took three.
template <bool PY>
__global__ __launch_bounds__(kWave) void k_flush1(Pool pool, Trees tr, EvalCache cache, EvalCache apply_cache,
                                                  const float *__restrict__ policy, int64_t pld,
                                                  const float *__restrict__ value, int64_t vld,
                                                  const int32_t *__restrict__ rowbase, int per_copy, int do_apply,
                                                  unsigned long long *stats, HostLeaf *host_leaf, int32_t tag) {
    __shared__ __attribute__((aligned(16))) float s_row[84];
    if (do_apply) {
        apply_wave(pool, tr, apply_cache, policy, pld, value, vld, rowbase, per_copy,
                   stats ? stats + kKApply * kRow : nullptr, 0, s_row);
        wave_memory_fence();  // the descent reads the records the apply wrote
    }
    select_wave<PY>(pool, tr, cache, stats, 0, s_row, host_leaf, tag);
}

// One round of many trees in one launch (round 5, uttt_round_hash_async): wave t applies its tree's
// evaluation of the previous round (k_apply's body, the slot from k_scan's slot_of) and then runs the
// tree's next descent (k_select's body). Trees are independent but for the evaluation cache, whose
// versioned records make a probe racing another tree's insert see either the old or the new record, and a
// hit or a miss give the same tree (a miss is evaluated later with the same values). One dispatch where
// k_apply and k_select took two.
template <bool PY>
__global__ __launch_bounds__(kBlock, 4) void k_round(Pool pool, Trees tr, EvalCache cache,
                                                  const float *__restrict__ policy, int64_t pld,
                                                  const float *__restrict__ value, int64_t vld,
                                                  unsigned long long *stats) {
    __shared__ __attribute__((aligned(16))) float s_row[kWavesPerBlock][84];
    const int t = wave_index();
    if (t >= tr.n_trees) return;
    const int slot = __builtin_amdgcn_readfirstlane(tr.slot_of[t]);
    if (slot >= 0) {
        apply_wave(pool, tr, cache, policy, pld, value, vld, nullptr, 0, stats ? stats + kKApply * kRow : nullptr,
                   slot, s_row[threadIdx.x >> 6]);
        wave_memory_fence();  // the descent reads the records the apply wrote
    }
    select_wave<PY>(pool, tr, cache, stats, t, s_row[threadIdx.x >> 6], nullptr, 0);
}

// The hash evaluator's outputs for one state into row `row` (k_hash_leaves' body): bit j = ch * 81 + R * 9 + C
// of the network input, as k_encode writes it, so the words and outputs are k_hash_eval's.
__device__ __forceinline__ void hash_leaf_row(const uttt_state_t &s, float *__restrict__ policy, float *__restrict__ value,
                                              int row);

// One tree-only round in ONE dispatch (round 6; UTTT_ROUND_DISPATCHES=3 keeps k_round +
// k_scan + k_hash_leaves). With the hash evaluator nothing needs the leaves in slot order, so the rows are
// indexed by TREE: wave t applies its tree's evaluation of the previous round from row t (apply != 0 and its
// pending word, still the previous round's, shows a queued leaf), runs the next descent (k_select's body), and
// evaluates the leaf it queued straight into row t. The round's counts, which k_scan produced, are summed
// per block into a partial (sc1 store) and the last block to arrive (striped arrival counters, then one top
// counter) adds the partials, publishes them (device counts, the host ring and its tag) and resets the
// counters for the next round. Every tree's work is k_round's in the same order, so every result is the
// three-dispatch round's (the fused-rounds test runs both).
constexpr int kR1Stripes = 8;
// uttt_rounds_hash_move's per-block count words: n0 (queued leaves) bits 0-4, n1 (budget stops) 5-9, n2
// (trees with simulations left) 10-14, at most kWavesPerBlock = 16 each; the round's tag (17 bits) above
constexpr int kPartTagShift = 15;
constexpr uint32_t kPartTagMask = 0x1FFFFu;
constexpr uint32_t kPartLiveMask = 0x1Fu | (0x1Fu << 10);
static_assert(kWavesPerBlock <= 31, "k_round1's per-block count words hold 5-bit counts");
constexpr int kR1Partial = 64;  // rctl: [0..7] stripe arrivals, [32] top, [64 + block] partials
template <bool PY>
__global__ __launch_bounds__(kBlock, 4) void k_round1(Pool pool, Trees tr, EvalCache cache, const float *apply_policy,
                                                   const float *apply_value, float *__restrict__ policy,
                                                   float *__restrict__ value, int apply, unsigned long long *stats,
                                                   int32_t *host_count, int32_t tag, uint32_t *rctl,
                                                   uint32_t *part_host, uint32_t *part_dev, const uint32_t *part_prev,
                                                   int nb_prev, int stats_parity) {
    __shared__ __attribute__((aligned(16))) float s_row[kWavesPerBlock][84];
    __shared__ uint32_t s_cnt;
    __shared__ int s_last;
    // part_host (uttt_rounds_hash_move's rounds, no kernel timing): no last-block publish. Each block stores its
    // counts with the round's tag into its own word of a host array (and of a device array the next round's
    // empty-round check reads, part_prev), and the host sums the words once every block's has the tag: the
    // arrival atomics, the partials' reload and the last block's drain left each round's critical path (round 6)
    if (part_host) {
        if (stats && blockIdx.x == 0 && threadIdx.x < kWave) {
            // the previous round's slowest tree (the other parity's rows) into the sums; this round's waves
            // write this parity's rows meanwhile
            const int rm = stats_parity ? kKSelMax : kKSelMaxB, rt = stats_parity ? kKSelTripMax : kKSelTripMaxB;
            unsigned long long ml = 0ull, mt = 0ull;
            if (threadIdx.x < kStripes) {
                unsigned long long *a = stats + rm * kRow + threadIdx.x * kStripeStride;
                unsigned long long *bb = stats + rt * kRow + threadIdx.x * kStripeStride;
                ml = __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                mt = __hip_atomic_load(bb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(a, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(bb, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                const unsigned long long ol = __shfl_xor(ml, off), ot = __shfl_xor(mt, off);
                ml = ol > ml ? ol : ml;
                mt = ot > mt ? ot : mt;
            }
            if (threadIdx.x == 0) {
                stats[kKSelMaxSum * kRow] += ml;
                stats[kKSelTripMaxSum * kRow] += mt;
            }
        }
        const uint32_t t17 = ((uint32_t)tag & kPartTagMask) << kPartTagShift;
        bool empty = false;
        if (part_prev) {  // the previous round queued no leaf and left no tree with simulations
            bool busy = false;
            for (int i = threadIdx.x; i < nb_prev; i += kBlock) busy |= (part_prev[i] & kPartLiveMask) != 0u;
            empty = !__syncthreads_or(busy);
        }
        if (empty) {
            if (threadIdx.x == 0) {
                part_dev[blockIdx.x] = t17;
                __hip_atomic_store(part_host + blockIdx.x, t17, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            return;
        }
    }
    // a round behind one that queued no leaf and left no tree with simulations (the host's look-ahead rounds
    // past a move's end) has nothing to apply or select: every pending word is already 0 and the counts
    // stay 0, so block 0 publishes them and its tag, and every other block leaves at once (round 6: such a
    // round cost ~19 us of GPU time as a full pass over the trees; k_begin marks a new search non-empty)
    if (!part_host && tr.count[0] == 0 && tr.count[2] == 0) {
        if (blockIdx.x == 0 && threadIdx.x == 0 && host_count) {
            st_host(host_count + 0, 0);
            st_host(host_count + 1, 0);
            st_host(host_count + 2, 0);
            host_stores_done();
            st_host(host_count + 3, tag);
        }
        return;
    }
    const int t = wave_index();
    const int lane = lane_id();
    if (threadIdx.x == 0) s_cnt = 0u;
    __syncthreads();
    CachePublish held{-1, 0u};  // the apply's cache insert, published after this block's drain below
    if (t < tr.n_trees) {
        const int prev = __builtin_amdgcn_readfirstlane(tr.pending[t]);  // the previous round's, until the select
        if (apply && (prev & 1)) {
            apply_wave(pool, tr, cache, apply_policy, 81, apply_value, 1, nullptr, 0,
                       stats ? stats + kKApply * kRow : nullptr, t, s_row[threadIdx.x >> 6], t, prev >> 8, nullptr,
                       false, &held);
            wave_memory_fence();  // the descent reads the records the apply wrote
        }
        uttt_state_t leaf;
        const int p = select_wave<PY>(pool, tr, cache, stats, t, s_row[threadIdx.x >> 6], nullptr, 0,
                                      part_host ? stats_parity : 0, &leaf);
        if (p & 1) hash_leaf_row(leaf, policy, value, t);  // the queued leaf (its state from the descent)
        const int q = p & 0xFF;
        if (lane == 0)  // pending | stopped << 10 | left << 20 (at most kWavesPerBlock each)
            atomicAdd(&s_cnt, (uint32_t)((q == 1 || q == 3) ? 1 : 0) | ((q == 2 ? 1u : 0u) << 10) |
                                  ((q >= 2 ? 1u : 0u) << 20));
    }
    // every wave's stores (rows, records, stats atomics, a held cache record) complete before the block's
    // partial is published, and before the held record's flag
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    cache_publish(cache, held);
    __syncthreads();
    if (part_host) {  // the block's counts and the round's tag, one word (its stores drained above)
        if (threadIdx.x == 0) {
            const uint32_t w = (((uint32_t)tag & kPartTagMask) << kPartTagShift) | ((s_cnt >> 20) << 10) |
                               (((s_cnt >> 10) & 0x3FFu) << 5) | (s_cnt & 0x3FFu);
            part_dev[blockIdx.x] = w;
            __hip_atomic_store(part_host + blockIdx.x, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        return;
    }
    const int nb = (int)gridDim.x, b = (int)blockIdx.x;
    if (threadIdx.x == 0) {
        __hip_atomic_store(rctl + kR1Partial + b, s_cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int st = b & (kR1Stripes - 1);
        const uint32_t in_stripe = (uint32_t)((nb - st + kR1Stripes - 1) / kR1Stripes);
        const int stripes = nb < kR1Stripes ? nb : kR1Stripes;
        int last = 0;
        if (__hip_atomic_fetch_add(rctl + st, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == in_stripe - 1)
            last = __hip_atomic_fetch_add(rctl + 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                   (uint32_t)(stripes - 1);
        s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    // the last block: every partial was published before its block's arrival (sc1 loads, no stale L1 copy)
    uint32_t c0 = 0u, c1 = 0u, c2 = 0u;
    for (int i = threadIdx.x; i < nb; i += kBlock) {
        const uint32_t v = __hip_atomic_load(rctl + kR1Partial + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        c0 += v & 0x3FFu;
        c1 += (v >> 10) & 0x3FFu;
        c2 += v >> 20;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        c0 += __shfl_xor(c0, off);
        c1 += __shfl_xor(c1, off);
        c2 += __shfl_xor(c2, off);
    }
    __shared__ uint32_t s_sum[3][kWavesPerBlock];
    if (lane == 0) {
        s_sum[0][threadIdx.x >> 6] = c0;
        s_sum[1][threadIdx.x >> 6] = c1;
        s_sum[2][threadIdx.x >> 6] = c2;
    }
    // the select's slowest tree (as k_scan folds it): the max over the stripes, one per lane of wave 1
    if (stats && threadIdx.x >= kWave && threadIdx.x < 2 * kWave) {
        const int l = threadIdx.x - kWave;
        unsigned long long ml = 0ull, mt = 0ull;
        if (l < kStripes) {
            unsigned long long *a = stats + kKSelMax * kRow + l * kStripeStride;
            unsigned long long *bb = stats + kKSelTripMax * kRow + l * kStripeStride;
            ml = __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            mt = __hip_atomic_load(bb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(bb, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const unsigned long long ol = __shfl_xor(ml, off), ot = __shfl_xor(mt, off);
            ml = ol > ml ? ol : ml;
            mt = ot > mt ? ot : mt;
        }
        if (l == 0) {
            stats[kKSelMaxSum * kRow] += ml;
            stats[kKSelTripMaxSum * kRow] += mt;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int n0 = 0, n1 = 0, n2 = 0;
        for (int w = 0; w < kWavesPerBlock; ++w) {
            n0 += (int)s_sum[0][w];
            n1 += (int)s_sum[1][w];
            n2 += (int)s_sum[2][w];
        }
        tr.count[0] = n0;
        tr.count[1] = n1;
        tr.count[2] = n2;
        for (int i = 0; i < kR1Stripes; ++i) rctl[i] = 0u;
        rctl[32] = 0u;
        if (host_count) {
            __hip_atomic_store(host_count + 0, n0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(host_count + 1, n1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(host_count + 2, n2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            host_stores_done();
            st_host(host_count + 3, tag);
        }
    }
}

// A one-dispatch round's staged evaluation applied by tree (flush before anything else reads the trees)
__global__ __launch_bounds__(kBlock) void k_apply_tree(Pool pool, Trees tr, EvalCache cache, const float *policy,
                                                       const float *value, unsigned long long *bytes_ctr) {
    __shared__ __attribute__((aligned(16))) float s_row[kWavesPerBlock][84];
    const int t = wave_index();
    if (t >= tr.n_trees) return;
    const int prev = __builtin_amdgcn_readfirstlane(tr.pending[t]);
    if (prev & 1)
        apply_wave(pool, tr, cache, policy, 81, value, 1, nullptr, 0, bytes_ctr, t, s_row[threadIdx.x >> 6], t,
                   prev >> 8);
}

// -------------------------------------------------------------- hash eval --
// Deterministic test evaluator on the NCHW rows: one wave per row; the 4
// ballots of "x != 0" over the 243 floats are exactly the 4 hash words.
__global__ __launch_bounds__(kBlock) void k_hash_eval(const float *__restrict__ x, int n, float *__restrict__ policy,
                                                      float *__restrict__ value) {
    const int lane = lane_id();
    const int row = wave_index();
    if (row >= n) return;
    const float *xr = x + (size_t)row * 243;
    uint64_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int j = i * 64 + lane;
        w[i] = __ballot(j < 243 && xr[j] != 0.0f);
    }
    const uint64_t h = hash_words(w);
    policy[(size_t)row * 81 + lane] = hash_prior(h, lane);
    if (lane < 17) policy[(size_t)row * 81 + 64 + lane] = hash_prior(h, 64 + lane);
    if (lane == 0) value[row] = hash_value(h);
}

// ---------------------------------------------------------- root results --
__device__ __forceinline__ int root_children(const Pool &pool, size_t base, int &first) {
    const uint4 r = pool.rec[base];
    first = link_first(r.w);
    return meta_L(r.z);
}
__device__ __forceinline__ int visits_of(const Pool &pool, size_t i) { return meta_n(pool.rec[i].z); }

// pv_mcts_scores' return value (uttt_mcts.cpp:177-195): root child visits as
// f32 -> one-hot first max (t == 0) or boltzman (:199-216).
__device__ void root_scores(const Pool &pool, size_t base, float temperature, float *sc, int &L) {
    int first;
    L = root_children(pool, base, first);
    if (temperature == 0.0f) {
        int mi = 0;
        float mv = L ? (float)visits_of(pool, base + first) : 0.0f;
        for (int i = 1; i < L; ++i) {
            const float v = (float)visits_of(pool, base + first + i);
            if (v > mv) {
                mv = v;
                mi = i;
            }
        }
        for (int i = 0; i < L; ++i) sc[i] = (i == mi) ? 1.0f : 0.0f;
    } else {
        // glibc's powf (what the reference's std::pow(float, float) calls) evaluates in
        // double and rounds once; ocml's f32 powf is not correctly rounded (pow(19, 1)
        // came out 1 ulp low), so do the same: double pow of the f32 operands, one rounding.
        const double y = (double)(1.0f / temperature);
        float sum = 0.0f;
        for (int i = 0; i < L; ++i) {
            sc[i] = (float)pow((double)visits_of(pool, base + first + i), y);
            sum += sc[i];
        }
        if (sum > 0)
            for (int i = 0; i < L; ++i) sc[i] /= sum;
    }
}

// The same evaluator on this round's pending leaves straight from their states (the device-count
// rounds: no NCHW input is written): bit j = ch * 81 + R * 9 + C of the network input, as k_encode
// writes it, so the words and outputs are k_hash_eval's. One wave per slot; the count is read on the
// device (the grid covers every tree).
__global__ __launch_bounds__(kBlock) void k_hash_leaves(Trees tr, float *__restrict__ policy,
                                                        float *__restrict__ value) {
    const int row = wave_index();
    if (row >= tr.count[0]) return;
    const uttt_state_t s = tr.leaf[tr.tree_of[row]];
    hash_leaf_row(s, policy, value, row);
}

__device__ __forceinline__ void hash_leaf_row(const uttt_state_t &s, float *__restrict__ policy, float *__restrict__ value,
                                              int row) {
    const int lane = lane_id();
    uint32_t m[3];
    legal_mask(s, m);
    uint64_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int j = i * 64 + lane;
        bool on = false;
        if (j < 243) {
            const int ch = j / 81, a = action_at(j % 81);
            on = (ch == 0 ? bit_of(s.own, a) : (ch == 1 ? bit_of(s.opp, a) : bit_of(m, a))) != 0u;
        }
        w[i] = __ballot(on);
    }
    const uint64_t h = hash_words(w);
    policy[(size_t)row * 81 + lane] = hash_prior(h, lane);
    if (lane < 17) policy[(size_t)row * 81 + 64 + lane] = hash_prior(h, 64 + lane);
    if (lane == 0) value[row] = hash_value(h);
}

__global__ void k_root_visits(Pool pool, Trees tr, int32_t *visits, int32_t *n_legal) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= tr.n_trees * 81) return;
    const int t = g / 81, i = g % 81;
    const size_t base = (size_t)t * pool.cap;
    int first;
    const int L = root_children(pool, base, first);
    visits[g] = i < L ? visits_of(pool, base + first + i) : 0;
    if (i == 0) n_legal[t] = L;
}

__global__ void k_root_scores(Pool pool, Trees tr, float temperature, float *scores, int32_t *n_legal) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= tr.n_trees) return;
    float *sc = scores + (size_t)t * 81;  // the output row is the working buffer (no scratch)
    int L;
    root_scores(pool, (size_t)t * pool.cap, temperature, sc, L);
    for (int i = L; i < 81; ++i) sc[i] = 0.0f;
    n_legal[t] = L;
}

// ------------------------------------------------- resident one-tree search --
// A whole one-tree search as ONE resident wave (round 6; uttt_search1_*): the reference's
// pv_mcts_scores (uttt_mcts.cpp:84-196) driven through python_bindings.cpp:11-47 calls the model once per
// flush, so the search needs the host between flushes; instead of a launch per flush (k_flush1), the wave
// stays resident and meets the host through fine-grained pinned memory (Search1Host): it writes the flush's
// leaf, its copies and a sequence tag (system-scope release), polls for the host's command (the evaluation
// rows the host wrote beside it, then the command's sequence), applies them (k_apply's body) and descends
// to the next leaf (k_select's body); when the tree has no simulation left it computes the root's scores
// (k_root_scores' body) into host memory and exits. Same tree, same order of operations as k_begin +
// k_flush1 + k_root_scores, so the same results. Exit conditions every path reaches: the search's end, the
// host's exit word, and 100 ms without a command (s_memrealtime at 100 MHz); after a timeout the host
// relaunches the wave in resume mode (the command it wrote is applied first).
struct Search1Host {
    // device -> host
    int32_t tag, count, k, status;  // a leaf (count 1) or the end (count 0); status: the tree's error bits
    int32_t n_legal, gone, pad0, pad1;  // gone: the command sequence the wave timed out waiting for (0: none)
    // the wave's time split (s_memrealtime ticks of 10 ns, this launch): descents, applies, waits for the host
    int32_t t_select, t_apply, t_wait, pad3;
    uttt_state_t leaf;
    float scores[84];  // 81 used
    // host -> device: the command, sequence (low word) and rows (high word) in one 8-byte store the wave
    // reads whole; the exit word
    uint64_t cmd;
    int32_t cmd_exit, pad2;
    // the evaluation rows: policy [rows][96] (81 used), value [rows] (one leaf: its row base is 0)
};
static_assert(offsetof(Search1Host, cmd) % 8 == 0, "Search1Host::cmd must be 8-byte aligned");

constexpr int kSearch1Timeout = 10000000;  // 100 ms of s_memrealtime (100 MHz)

template <bool PY>
__global__ __launch_bounds__(kWave) void k_search1(Pool pool, Trees tr, EvalCache cache, uttt_state_t root,
                                                   float temperature, Search1Host *hs, const float *policy,
                                                   const float *value, int32_t seq, int32_t resume) {
    __shared__ __attribute__((aligned(16))) float s_row[84];
    __shared__ int32_t s_rowbase;  // the flush's first row: 0 (in LDS, not a PCIe round trip per apply)
    __shared__ __attribute__((aligned(16))) float s_copies[8 * 84];  // per-copy rows' prior sums (apply_wave)
    const int lane = lane_id();
    if (lane == 0) s_rowbase = 0;
    if (!resume) {  // k_begin's body for tree 0 (root expanded with uniform priors; py semantics: plain root)
        uint32_t m[3];
        legal_mask(root, m);
        if (tr.py) {
            const bool any = __ballot(bit_of(m, lane) != 0u) != 0ull || __ballot(lane < 17 && bit_of(m, 64 + lane) != 0u);
            if (lane == 0) {
                pool.rec[0] = make_uint4(0u, 0u, make_meta(kNoAction, 0u), 0u);
                tr.root[0] = root;
                TreeCtl c;
                c.sims_done = 0;
                c.node_count = 1;
                c.status = any ? kLive : 0;
                c.pad = 0;
                tr.ctl[0] = c;
            }
        } else {
            const bool l0 = bit_of(m, lane) != 0u;
            const bool l1 = lane < 17 && bit_of(m, 64 + lane) != 0u;
            const uint64_t b0 = __ballot(l0), b1 = __ballot(l1);
            const int L = __popcll(b0) + __popcll(b1);
            const float up = L ? 1.0f / (float)L : 0.0f;
            if (l0) pool.rec[1 + __popcll(b0 & lanes_below())] = new_child(up, (uint32_t)lane);
            if (l1) pool.rec[1 + __popcll(b0) + __popcll(b1 & lanes_below())] = new_child(up, (uint32_t)(64 + lane));
            if (lane == 0) {
                pool.rec[0] = make_uint4(0u, 0u, make_meta(kNoAction, (uint32_t)L), make_link(L ? 1u : 0u, L ? 1u : 0u));
                tr.root[0] = root;
                TreeCtl c;
                c.sims_done = 0;
                c.node_count = 1 + L;
                c.status = L > 0 ? kLive : 0;
                c.pad = 0;
                tr.ctl[0] = c;
            }
        }
        wave_memory_fence();
    }
    bool apply = resume != 0;  // resume: the command of sequence `seq` is waiting in host memory
    int rows = resume ? (int)__builtin_amdgcn_readfirstlane((int)(
                            __hip_atomic_load(&hs->cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >> 32))
                      : 0;
    uint64_t tk_sel = 0, tk_apply = 0, tk_wait = 0, tk = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (apply) {
            // per-copy rows bypass the evaluation cache (as host_apply_args)
            EvalCache acache = cache;
            if (rows > 1) acache.flag = nullptr;
            apply_wave(pool, tr, acache, policy, 96, value, 1, &s_rowbase, rows > 1 ? 1 : 0, nullptr, 0, s_row, 0,
                       __builtin_amdgcn_readfirstlane(tr.pending[0]) >> 8, s_copies, true);
            wave_memory_fence();  // the descent reads the records the apply wrote
            const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
            tk_apply += t1 - tk;
            tk = t1;
        }
        const int p = select_wave<PY>(pool, tr, cache, nullptr, 0, s_row, nullptr, 0);
        const int q = p & 0xFF;
        {
            const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
            tk_sel += t1 - tk;
            tk = t1;
        }
        if (q == 2) {  // stopped by the select budget before a leaf: descend again (as uttt_search_select_host)
            apply = false;
            continue;
        }
        ++seq;
        if (q == 1 || q == 3) {  // a leaf: hand it to the host
            wave_memory_fence();
            // the leaf (lanes 0-7, one store), its copies, the count and the time split, then the tag
            const int32_t lw = reinterpret_cast<const int32_t *>(&tr.leaf[0])[lane & 7];
            if (lane < 8) st_host(reinterpret_cast<int32_t *>(&hs->leaf) + lane, lw);
            if (lane == 0) {
                st_host(&hs->k, tr.rec[0].k);
                st_host(&hs->t_select, (int32_t)tk_sel);
                st_host(&hs->t_apply, (int32_t)tk_apply);
                st_host(&hs->t_wait, (int32_t)tk_wait);
                st_host(&hs->count, 1);
            }
            host_stores_done();
            if (lane == 0) st_host(&hs->tag, seq);
            // wait for the host's command of this sequence (its rows were written before it; they are read
            // with system-coherent loads, so the poll needs no acquire and its cache invalidation)
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            int got = 0;
            for (;;) {
                uint64_t c = 0;
                int x = 0;
                if (lane == 0) {
                    c = __hip_atomic_load(&hs->cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    x = __hip_atomic_load(&hs->cmd_exit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                const int cs = __builtin_amdgcn_readfirstlane((int)(uint32_t)c);
                x = __builtin_amdgcn_readfirstlane(x);
                if (cs == seq) {
                    rows = __builtin_amdgcn_readfirstlane((int)(c >> 32));
                    got = 1;
                    break;
                }
                if (x) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > (uint64_t)kSearch1Timeout) {
                    if (lane == 0) st_host(&hs->gone, seq);
                    host_stores_done();
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (!got) return;
            const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
            tk_wait += t1 - tk;
            tk = t1;
            apply = true;
            continue;
        }
        // the search's end: the root's scores (k_root_scores' body) and the tree's status, then the tag
        wave_memory_fence();
        int L = 0;
        if (lane == 0) root_scores(pool, 0, temperature, s_row, L);  // the LDS row as the working buffer
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        L = __builtin_amdgcn_readfirstlane(L);
        for (int i = lane; i < 81; i += kWave) st_host(&hs->scores[i], i < L ? s_row[i] : 0.0f);
        if (lane == 0) {
            st_host(&hs->n_legal, L);
            st_host(&hs->t_select, (int32_t)tk_sel);
            st_host(&hs->t_apply, (int32_t)tk_apply);
            st_host(&hs->t_wait, (int32_t)tk_wait);
            st_host(&hs->status, (int32_t)(tr.ctl[0].status & kErrMask));
            st_host(&hs->count, 0);
        }
        host_stores_done();
        if (lane == 0) st_host(&hs->tag, seq);
        return;
    }
}

// -------------------------------------------------------------- self-play --
struct Slot {
    uttt_state_t state;
    int64_t game;        // game id being played (-1: none)
    int32_t ply;
    int32_t live;
    int32_t finished;    // set by k_move_end when the game just ended
    int32_t fin_len;
    int64_t fin_game;
    int64_t fin_offset;  // arena row of its first ply
    int32_t fin_value;   // value of ply 0 (self_play_cpp.py:95)
    int32_t seed_pending;  // 1: k_finalize gave the slot a new game whose MT19937 key k_archive seeds
};

static_assert(offsetof(Slot, ply) == 40 && offsetof(Slot, live) == 44 && offsetof(Slot, finished) == 48 &&
                  offsetof(Slot, fin_len) == 52,
              "k_finalize reads Slot bytes 40..55 as one int4 (ply, live, finished, fin_len)");

struct GameEntry {
    int64_t game;
    int64_t offset;
    int64_t length;
};

struct SelfPlay {
    Slot *slot;
    uint32_t *mt_key;      // [slot][624]
    int32_t *mt_pos;       // [slot]
    uttt_state_t *ply_state;  // [slot][81]
    double *ply_policy;    // [slot][81][81]
    int8_t *ply_action;    // [slot][81]
    uttt_state_t *ar_state;
    double *ar_policy;
    int8_t *ar_action;
    int8_t *ar_value;
    GameEntry *games;
    int64_t *ctr;          // [0] next game id, [1] games finished, [2] arena plies used
    int32_t *live;         // [slot] flags for k_begin
    int32_t *work;         // [1 + slot]: k_finalize's count, then the slots k_archive has work for
    int64_t game_end;
    int64_t arena_cap;
    int64_t games_cap;
    uint32_t seed_base;
    float temperature;
    int32_t slots;
};

// numpy legacy RandomState: init_genrand(seed) (mt19937_seed), genrand_int32
// with the standard twist/tempering, random_sample = 53-bit double of 2 draws.
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

// The standard twist of one 624-word key by the 64 lanes of a wave. Element i reads key[i], key[i + 1]
// (old; key[0] new for i = 623) and key[(i + 397) % 624] (old for i < 227, new beyond), so three
// stages, [0, 227), [227, 454), [454, 624), each lane loading all its inputs before any store, run the
// sequential loop's exact updates (a thread's 624 dependent round trips took most of k_move_end).
__device__ void mt_twist_wave(uint32_t *key) {
    const int lane = lane_id();
    constexpr int lo[3] = {0, 227, 454}, hi[3] = {227, 454, 624};
#pragma unroll
    for (int st = 0; st < 3; ++st) {
        uint32_t a[4], b[4], c[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = lo[st] + lane + 64 * j;
            if (i < hi[st]) {
                a[j] = key[i];
                b[j] = key[i + 1 < 624 ? i + 1 : 0];
                c[j] = key[i + 397 < 624 ? i + 397 : i + 397 - 624];
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = lo[st] + lane + 64 * j;
            if (i < hi[st]) {
                const uint32_t y = (a[j] & 0x80000000u) | (b[j] & 0x7fffffffu);
                uint32_t v = c[j] ^ (y >> 1);
                if (y & 1u) v ^= 0x9908b0dfu;
                key[i] = v;
            }
        }
        wave_memory_fence();  // this stage's words before the next stage reads them (other lanes)
    }
}

// np.add.reduce on a contiguous float64 vector (pairwise, 8 accumulators, blocks <= 128).
__device__ double np_sum(const double *a, int n, int stride) {
    if (n < 8) {
        double r = 0.0;
        for (int i = 0; i < n; ++i) r += a[i * stride];
        return r;
    }
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = a[j * stride];
    int i = 8;
    for (; i < n - (n % 8); i += 8)
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] += a[(i + j) * stride];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i * stride];
    return res;  // n <= 81 < 128: a single pairwise block
}

// A float held by lane i of the wave (i uniform), to every lane.
__device__ __forceinline__ float lane_float(float x, int i) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), i));
}

// One wave per slot: the per-move tail of self_play_cpp.play (:63-92). Entry i of the root's score
// row lives in lane i (x0) and lane i - 64 (x1); what is order-free (the arg-max, the f32 sum of
// integer visit counts) is a wave reduction, what is not (np.sum's pairwise blocks, the cumsum of
// np.random.choice) runs the reference's additions in its order on the wave's LDS copy of the row, the
// same in every lane (round 5: on v_readlane operands; round 3's thread-per-slot form walked the row in
// LDS, 81-step dependent chains per pass with one wave per 64 slots).
// fail (the asynchronous form: the search's failure flag, Trees::count[3]): on a failure this move's end
// changes nothing (no draw, no record, no refill), as the blocking form refuses before it runs
__global__ __launch_bounds__(kBlock) void k_move_end(Pool pool, SelfPlay sp, const int32_t *fail) {
    const int lane = lane_id();
    const int s = wave_index();
    if (s >= sp.slots) return;
    // the loads that do not depend on each other are issued together (round 6: the failure word, the slot,
    // the key position and the root's record were four dependent round trips before the first draw)
    const size_t base = (size_t)s * pool.cap;
    const int32_t failed = fail ? *fail : 0;
    Slot sl = sp.slot[s];
    int32_t pos = sp.mt_pos[s];
    int first;
    const int L = root_children(pool, base, first);
    if (failed) return;
    sl.finished = 0;
    if (!sl.live) {
        if (lane == 0) sp.slot[s] = sl;
        return;
    }
    // np.random.choice's random_sample (numpy legacy: two 32-bit draws, 53-bit double); a key that
    // runs out is twisted by the wave (mt_twist_wave)
    uint32_t *key = sp.mt_key + (size_t)s * 624;
    const bool h0 = lane < L, h1 = lane + 64 < L;
    const int n0 = h0 ? visits_of(pool, base + first + lane) : 0;
    const int n1 = h1 ? visits_of(pool, base + first + lane + 64) : 0;
    uint32_t w1, w2;
    if (pos >= 623) {
        const uint32_t k623 = key[623];
        mt_twist_wave(key);
        if (pos == 623) {  // the first word was key[623] before the twist
            w1 = mt_temper(k623);
            w2 = mt_temper(key[0]);
            pos = 1;
        } else {
            w1 = mt_temper(key[0]);
            w2 = mt_temper(key[1]);
            pos = 2;
        }
    } else {
        w1 = mt_temper(key[pos]);
        w2 = mt_temper(key[pos + 1]);
        pos += 2;
    }
    const double u = ((double)(w1 >> 5) * 67108864.0 + (double)(w2 >> 6)) / 9007199254740992.0;
    const int ply = sl.ply;
    // root visit counts (uttt_mcts.cpp:177-192, as root_scores): entry i in lane i / i - 64 (loaded above)
    double x0, x1;
    if (sp.temperature == 0.0f) {
        // one-hot first max: the largest count, then the lowest index holding it (counts < 2^24, so
        // the f32 compares of the reference order them as the integers do)
        int kk = max(h0 ? (n0 << 8) | (255 - lane) : -1, h1 ? (n1 << 8) | (255 - 64 - lane) : -1);
#pragma unroll
        for (int o = 32; o; o >>= 1) kk = max(kk, __shfl_xor(kk, o));
        const int mi = kk < 0 ? 0 : 255 - (kk & 0xFF);
        x0 = (h0 && lane == mi) ? 1.0 : 0.0;
        x1 = (h1 && lane + 64 == mi) ? 1.0 : 0.0;
    } else {
        const double y = (double)(1.0f / sp.temperature);  // glibc powf: double pow, one rounding
        float v0 = 0.0f, v1 = 0.0f, sum = 0.0f;
        if (y == 1.0) {
            // pow(x, 1) == x exactly (IEEE 754); a sum of integers below 2^24 is exact in f32 in
            // any order, so the reference's sequential sum is the wave's integer sum
            v0 = (float)n0;
            v1 = (float)n1;
            int t = n0 + n1;
#pragma unroll
            for (int o = 32; o; o >>= 1) t += __shfl_xor(t, o);
            sum = (float)t;
        } else {
            if (h0) v0 = (float)pow((double)n0, y);
            if (h1) v1 = (float)pow((double)n1, y);
            for (int i = 0; i < L; ++i) sum += i < 64 ? lane_float(v0, i) : lane_float(v1, i - 64);
        }
        if (sum > 0) {
            v0 = v0 / sum;
            v1 = v1 / sum;
        }
        x0 = (double)v0;
        x1 = (double)v1;
    }
    // The row's entries for the sequential f64 sums below go through this wave's LDS row (entry i at xr[i],
    // read at a uniform address): a load and an add per entry, where the v_readlane pair, the select of the
    // half and the prefix's lane select per entry made the move end VALU-issue bound (round 6; every lane
    // still runs the same additions in the same order)
    __shared__ double s_xrow[kWavesPerBlock][81];
    double *const xr = s_xrow[threadIdx.x >> 6];
    auto stage = [&]() {
        if (h0) xr[lane] = x0;
        if (h1) xr[64 + lane] = x1;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every lane's stores before any lane's reads
    };
    stage();
    // scores -> float64, renormalised with np.sum (:74-78): np.add.reduce's pairwise block (8
    // accumulators over i = j mod 8, then the remainder), the same additions in every lane
    double tot;
    if (L < 8) {
        tot = 0.0;
        for (int i = 0; i < L; ++i) tot += xr[i];
    } else {
        double r[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = xr[j];
        int i = 8;
        for (; i < L - (L % 8); i += 8)
#pragma unroll
            for (int j = 0; j < 8; ++j) r[j] += xr[i + j];
        tot = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < L; ++i) tot += xr[i];
    }
    x0 = h0 ? ((tot == 0.0) ? 1.0 / (double)L : x0 / tot) : 0.0;
    x1 = h1 ? ((tot == 0.0) ? 1.0 / (double)L : x1 / tot) : 0.0;
    stage();
    // np.random.choice(legal, p=d) (:86): cdf = cumsum; cdf /= cdf[-1]; searchsorted right. The
    // cumsum's prefixes are written over the row in place and land in the lanes of their entries; its last
    // prefix is cdf[-1].
    double acc = 0.0;
    for (int i = 0; i < L; ++i) {
        acc += xr[i];
        xr[i] = acc;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const double c0 = h0 ? xr[lane] : 0.0, c1 = h1 ? xr[64 + lane] : 0.0;
    const uint64_t b0 = __ballot(h0 && !(c0 / acc <= u)), b1 = __ballot(h1 && !(c1 / acc <= u));
    const int k = b0 ? __builtin_ctzll(b0) : (b1 ? 64 + __builtin_ctzll(b1) : L - 1);  // idx >= L -> L - 1
    // policy target (:81-83): entry i of the row goes to the i-th legal action, the rest are zero
    uint32_t m[3];
    legal_mask(sl.state, m);
    double *const row = sp.ply_policy + ((size_t)s * kMaxPlies + ply) * 81;
    int action = -1;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        const int a = lane + 64 * half;
        int rank = 0;
        bool legal = false;
        if (a < 81) {
            const int w = a / 27, b = a % 27;
            legal = (m[w] >> b) & 1u;
            rank = __builtin_popcount(m[w] & ((1u << b) - 1u));
            for (int q = 0; q < w; ++q) rank += __builtin_popcount(m[q]);
        }
        const double e0 = __shfl(x0, rank & 63), e1 = __shfl(x1, rank & 63);
        if (a < 81) row[a] = legal ? (rank < 64 ? e0 : e1) : 0.0;
        const uint64_t hit = __ballot(legal && rank == k);
        if (hit) action = 64 * half + __builtin_ctzll(hit);
    }
    if (lane == 0) {
        sp.mt_pos[s] = pos;
        sp.ply_state[(size_t)s * kMaxPlies + ply] = sl.state;
        sp.ply_action[(size_t)s * kMaxPlies + ply] = (int8_t)action;
        sl.state = next_state(sl.state, action);
        sl.ply = ply + 1;
        if (is_done(sl.state) || sl.ply >= kMaxPlies) {
            sl.finished = 1;
            sl.fin_len = sl.ply;
            sl.fin_game = sl.game;
            sl.fin_value = is_lose(sl.state) ? -1 : 0;  // self_play_cpp.py:95
            sl.live = 0;
        }
        sp.slot[s] = sl;
    }
}

// One block: give finished games arena rows (slot order) and free slots the
// next game ids (slot order) — deterministic for a given slot count.
// host_move (optional, fine-grained pinned): the counters after this move end and the failure word,
// stored at system scope by the kernel itself (the asynchronous move end: no copies on the stream)
__device__ __forceinline__ void store_host_i64(int64_t *p, int64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// fail / ctl / err (the asynchronous form): when the search's failure flag is set, the first failed tree
// (lowest slot) and its status go to *err (k_archive skips then) and to host_move[4], and the move is not
// ended (k_move_end changed nothing); the status scan runs only on that rare path (round 6: a k_tree_err
// launch per move scanned every tree's status on the critical path)
__global__ __launch_bounds__(1024) void k_finalize(SelfPlay sp, const int32_t *fail, const TreeCtl *ctl,
                                                   unsigned long long *err, int64_t *host_move) {
    __shared__ unsigned long long wsum[32];
    __shared__ int s_work;  // entries of k_archive's work list
    __shared__ unsigned long long s_first;
    const int tid = threadIdx.x;
    // the counters are read before the scans (only this kernel writes them, after its last barrier): their
    // round trip overlaps the slots' instead of following the scans
    const int64_t arena0 = sp.ctr[2], games0 = sp.ctr[1], next0 = sp.ctr[0];
    const int per = (sp.slots + 1023) / 1024;
    const int b = tid * per, e = min(b + per, sp.slots);
    // the scans need a slot's live / finished / fin_len only: one 16-byte load of Slot bytes 40..55 per slot
    // (up to kFinPer per thread, all in flight together, kept for the second pass), and the second pass
    // reads and rewrites only the slots that change (a game just finished or the slot is free); every other
    // slot was brought up to date by k_move_end. Round 5: the single block read and wrote every 80-byte
    // slot through one CU (31 us per move at 4,096 slots). They go out with the failure word's load (round 6).
    constexpr int kFinPer = 4;
    int4 hot[kFinPer];
#pragma unroll
    for (int j = 0; j < kFinPer; ++j)
        if (b + j < e) hot[j] = *reinterpret_cast<const int4 *>(reinterpret_cast<const char *>(sp.slot + b + j) + 40);
    if (fail && *fail) {
        if (threadIdx.x == 0) s_first = ~0ull;
        __syncthreads();
        for (int t = threadIdx.x; t < sp.slots; t += blockDim.x) {
            const uint32_t st = (uint32_t)ctl[t].status;
            if (st & kErrMask) atomicMin(&s_first, ((unsigned long long)t << 32) | st);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            *err = s_first;
            if (host_move) store_host_i64(host_move + 4, (int64_t)s_first);
        }
        return;
    }
    auto hot_of = [&](int i) -> int4 {
        return i - b < kFinPer ? hot[i - b] : *reinterpret_cast<const int4 *>(reinterpret_cast<const char *>(sp.slot + i) + 40);
    };
    long long fl = 0;
    int fr = 0, fc = 0, first_changed = -1;
    for (int i = b; i < e; ++i) {
        const int4 h = hot_of(i);  // ply, live, finished, fin_len
        if (h.z) {
            fl += h.w;
            ++fc;
        }
        if (!h.y) ++fr;
        if (first_changed < 0 && (h.z || !h.y)) first_changed = i;
    }
    // the thread's first changing slot (usually its only one: ~1 in 40 per move) is loaded whole now, so its
    // round trip runs under the scan instead of after it
    Slot first_slot;
    if (first_changed >= 0) first_slot = sp.slot[first_changed];
    unsigned long long fl_tot, cnt_tot;
    unsigned long long fl_ex = (unsigned long long)fl, cnt_ex = (unsigned long long)fr | ((unsigned long long)fc << 32);
    block_scan2_1024(fl_ex, cnt_ex, &fl_tot, &cnt_tot, wsum);
    long long off = arena0 + (long long)fl_ex;
    int gi = (int)(games0 + (long long)(cnt_ex >> 32));
    int fi = (int)(cnt_ex & 0xFFFFFFFFull);
    const long long fin_total = (long long)fl_tot;
    const int free_total = (int)(cnt_tot & 0xFFFFFFFFull), fin_count = (int)(cnt_tot >> 32);
    if (tid == 0) s_work = 0;
    __syncthreads();
    for (int i = b; i < e; ++i) {
        const int4 h = hot_of(i);
        if (!h.z && h.y) continue;  // playing on: nothing here changes it
        Slot sl = i == first_changed ? first_slot : sp.slot[i];
        if (sl.finished) {
            if (off + sl.fin_len <= sp.arena_cap && gi < sp.games_cap) {
                sl.fin_offset = off;
                GameEntry ge;
                ge.game = sl.fin_game;
                ge.offset = off;
                ge.length = sl.fin_len;
                sp.games[gi] = ge;
            } else {
                sl.fin_offset = -1;  // arena full: host reports UTTT_ERR_CAPACITY
            }
            off += sl.fin_len;
            ++gi;
        }
        if (!sl.live) {
            const int64_t g = next0 + fi;
            ++fi;
            if (g < sp.game_end) {
                sl.state.own[0] = sl.state.own[1] = sl.state.own[2] = 0u;
                sl.state.opp[0] = sl.state.opp[1] = sl.state.opp[2] = 0u;
                sl.state.mains = 0u;
                sl.state.active = -1;
                sl.game = g;
                sl.ply = 0;
                sl.live = 1;
                // the key is seeded by k_archive (one block per slot, so the ~1 in 40 slots refilled per
                // move seed on their own CUs): 624 dependent steps and 624 strided stores per new game
                // on this kernel's single CU were most of its time (round 4)
                sl.seed_pending = 1;
            } else {
                sl.game = -1;
            }
        }
        sp.live[i] = sl.live;
        sp.slot[i] = sl;
        // k_archive's work: a finished game to copy to the arena, or a new game's key to seed (about 1 in
        // 40 slots per move, so k_archive runs a short list instead of a workgroup per slot)
        if ((sl.finished && sl.fin_offset >= 0) || sl.seed_pending) sp.work[1 + atomicAdd(&s_work, 1)] = i;
    }
    __syncthreads();  // every thread read sp.ctr before it is rewritten
    if (tid == 0) {
        sp.work[0] = s_work;
        sp.ctr[2] = arena0 + fin_total;
        sp.ctr[1] = games0 + fin_count;
        const int64_t nxt = next0 + free_total;
        sp.ctr[0] = nxt < sp.game_end ? nxt : sp.game_end;
        // live slots for the next move: those still playing plus the free ones given a game
        sp.ctr[3] = (int64_t)(sp.slots - free_total) + (sp.ctr[0] - next0);
        if (host_move) {
            for (int i = 0; i < 4; ++i) store_host_i64(host_move + i, sp.ctr[i]);
            store_host_i64(host_move + 4, (int64_t)~0ull);
        }
    }
}

// Copy each just-finished game's plies to its arena rows, with values
// (self_play_cpp.py:95-99: ply 0 gets the final value, then alternating), and seed the MT19937
// key of a slot k_finalize gave a new game (numpy's init_genrand(seed_base + game)).
// The seeding wave runs init_genrand's 624-step chain uniformly (every lane the same values, wave-uniform
// operands) and lane i & 63 keeps step i: ten coalesced 64-word stores instead of 624 one-lane stores.
// Round 6: the chain stays in SGPRs (the seed made wave-uniform) and each step's value goes to its lane by one
// v_writelane with an immediate lane index (steps unrolled by template), so a step is five scalar ops and one
// vector op (a compare and a select per step before: 18 us per seed, the move end's longest chain).
template <int J>
__device__ __forceinline__ uint32_t write_lane(uint32_t v, uint32_t x) {
    asm("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(x), "i"(J));
    return v;
}
template <int J, int N>
struct SeedSteps {  // init_genrand's steps base + J .. base + N - 1, step base + j into lane j
    static __device__ __forceinline__ void run(uint32_t &x, uint32_t &mine, uint32_t base) {
        x = 1812433253u * (x ^ (x >> 30)) + base + (uint32_t)J;
        mine = write_lane<J>(mine, x);
        SeedSteps<J + 1, N>::run(x, mine, base);
    }
};
template <int N>
struct SeedSteps<N, N> {
    static __device__ __forceinline__ void run(uint32_t &, uint32_t &, uint32_t) {}
};
__device__ __forceinline__ void mt_seed_wave(uint32_t *key, int32_t *pos, uint32_t seed) {
    static_assert(624 == 9 * kWave + 48, "init_genrand's 624 words as 9 full waves and 48");
    const int lane = lane_id();
    uint32_t x = (uint32_t)__builtin_amdgcn_readfirstlane((int)seed);
    uint32_t mine = x;  // key[0] = seed
    SeedSteps<1, kWave>::run(x, mine, 0u);
    key[lane] = mine;
    for (int i0 = kWave; i0 < 9 * kWave; i0 += kWave) {
        SeedSteps<0, kWave>::run(x, mine, (uint32_t)i0);
        key[i0 + lane] = mine;
    }
    SeedSteps<0, 48>::run(x, mine, 9u * kWave);
    if (lane < 48) key[9 * kWave + lane] = mine;
    if (lane == 0) *pos = 624;
}

// Each block: the slots of k_finalize's work list (entry w, w + grid, ...; round 6, in place of a workgroup
// per slot). A finished game's plies are copied with eight independent loads in flight per thread before
// their stores (round 4: one dependent load-store pair per iteration, ~19 memory round trips per game, a
// 39 us launch). seed: the last wave also seeds a refilled slot's key (selfplay_begin and the blocking move
// end, and the asynchronous one by default); UTTT_SEED_STREAM=1 runs the whole kernel on the engine's side
// stream, off the critical path (a key is first drawn from, and a finished game's rows first overwritten, at
// the next move's end).
constexpr int kArchiveBlocks = 256;
__global__ __launch_bounds__(256) void k_archive(SelfPlay sp, const unsigned long long *err, int seed) {
    // the failure word, the list's length and this block's first entry are loaded together (the grid is at
    // most the slot count and the list has room for every slot, so entry blockIdx.x is in bounds): one round
    // trip before the first slot load instead of three
    const unsigned long long e0 = err ? *err : ~0ull;
    const int n_work = sp.work[0];
    const int first = sp.work[1 + blockIdx.x];
    if (e0 != ~0ull) return;
    for (int w = blockIdx.x; w < n_work; w += gridDim.x) {
        const int s = w == (int)blockIdx.x ? first : sp.work[1 + w];
        const Slot sl = sp.slot[s];
        const int wave = (int)threadIdx.x >> 6;
        if (seed && sl.seed_pending && wave == 3) {
            mt_seed_wave(sp.mt_key + (size_t)s * 624, sp.mt_pos + s, sp.seed_base + (uint32_t)sl.game);
            if (lane_id() == 0) sp.slot[s].seed_pending = 0;
        }
        if (!sl.finished || sl.fin_offset < 0) continue;
        const size_t src0 = (size_t)s * kMaxPlies, dst0 = (size_t)sl.fin_offset;
        const double *__restrict__ from = sp.ply_policy + src0 * 81;
        double *__restrict__ to = sp.ar_policy + dst0 * 81;
        const int n = sl.fin_len * 81;  // the game's policy rows are contiguous in both places
        constexpr int kU = 8;
        for (int i0 = threadIdx.x; i0 < n; i0 += 256 * kU) {
            double v[kU];
#pragma unroll
            for (int j = 0; j < kU; ++j) v[j] = i0 + 256 * j < n ? from[i0 + 256 * j] : 0.0;
#pragma unroll
            for (int j = 0; j < kU; ++j)
                if (i0 + 256 * j < n) to[i0 + 256 * j] = v[j];
        }
        for (int ply = threadIdx.x; ply < sl.fin_len; ply += 256) {
            sp.ar_state[dst0 + ply] = sp.ply_state[src0 + ply];
            sp.ar_action[dst0 + ply] = sp.ply_action[src0 + ply];
            sp.ar_value[dst0 + ply] = (int8_t)((ply & 1) ? -sl.fin_value : sl.fin_value);
        }
    }
}

static int archive_grid(int slots) { return slots < kArchiveBlocks ? slots : kArchiveBlocks; }

__global__ void k_hwc(const uttt_state_t *st, int64_t n, float *out) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n * 81) return;
    const int64_t row = g / 81;
    const int a = (int)(g % 81);
    const uttt_state_t s = st[row];
    uint32_t m[3];
    legal_mask(s, m);
    float *o = out + row * 243 + image_index(a) * 3;
    o[0] = bit_of(s.own, a) ? 1.0f : 0.0f;
    o[1] = bit_of(s.opp, a) ? 1.0f : 0.0f;
    o[2] = bit_of(m, a) ? 1.0f : 0.0f;
}

}  // namespace uttt

// ============================================================== host side ==
using namespace uttt;

struct uttt_engine {
    int device = 0;
    int max_trees = 0;
    int max_sims = 0;
    int64_t cap = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    Pool pool{};
    Trees tr{};
    int32_t *h_count = nullptr;  // pinned
    int32_t *h_ring = nullptr;   // fine-grained pinned: kCountRing x {pending, stopped, left, tag}, k_scan-written
    HostLeaf *h_leaf = nullptr;  // fine-grained pinned: a one-tree round's result (uttt_search_select_host)
    float *h_eval = nullptr;     // fine-grained pinned: its evaluation, read by k_apply (uttt_search_apply_host):
                                 // [rows][96] policy, [rows] value, one int32 0 (the per-copy row base)
    int64_t h_eval_rows = 0;
    // a hash round's evaluation staged by uttt_round_hash_async, applied by the next round's k_round (or by
    // flush_dev_apply before any other call that reads the trees); UTTT_FUSED_ROUNDS=0: separate launches
    const float *dev_apply_policy = nullptr, *dev_apply_value = nullptr;
    bool dev_apply_staged = false;
    bool dev_apply_by_tree = false;  // staged by a one-dispatch round (k_round1): rows by tree, no scan
    // the resident one-tree search (uttt_search1_*, k_search1): its host block and evaluation rows
    Search1Host *h_s1 = nullptr;  // fine-grained pinned: Search1Host, then policy [cap][96], value [cap]
    int32_t s1_cap = 0, s1_seq = 0;
    bool s1_alive = false;  // a k_search1 wave may still be resident on the stream
    uttt_state_t s1_root{};
    float s1_temperature = 0.0f;
    uint32_t *d_r1ctl = nullptr;     // k_round1's arrival counters and per-block partials (zero between rounds)
    // uttt_rounds_hash_move's per-block count words: host [kCountRing][part_cap] (fine-grained pinned), device
    // [2][part_cap] (the previous round's, for the empty-round check)
    uint32_t *h_part = nullptr, *d_part = nullptr;
    int32_t part_cap = 0;
    uint32_t round_parity = 0;  // the per-block rounds' select-statistics parity (alternates every round)
    int32_t host_apply_rows = 0;  // a one-tree evaluation staged by uttt_search_apply_host, applied by the next
                                  // k_flush1 (or by flush_host_apply before any other call that reads the tree)
    int32_t leaf_tag = 0;
    int32_t *d_rowbase = nullptr;
    float *d_pol_scratch = nullptr;
    float *d_val_scratch = nullptr;
    int64_t scratch_rows = 0;
    float *d_scores = nullptr;
    int32_t *d_nlegal = nullptr;
    int32_t *d_visits = nullptr;
    int64_t bytes = 0;
    // round state
    int phase = 0;  // 0 idle, 1 search begun (select next), 2 selected (apply next),
                    // 3 selected without reading the count (uttt_search_select_async; apply next)
    int n_pending = 0;
    bool selfplay = false;
    // self-play
    SelfPlay sp{};
    int64_t sp_arena_used = 0;
    int64_t *h_move = nullptr;          // pinned: [0..3] sp.ctr after the last move end, [4] error word
    unsigned long long *d_err = nullptr;  // first failed tree of a move: (tree << 32) | status, or ~0
    // evaluation cache (off unless uttt_engine_set_cache)
    EvalCache cache{};
    int cache_log2 = 0;
    int cache_clear_every = 0;
    bool cache_owner = true;  // false: the table belongs to another engine (uttt_engine_share_cache)
    int64_t moves = 0;
    unsigned long long *d_cache_ctr = nullptr;
    // telemetry
    bool timing = false;
    unsigned long long *d_bytes = nullptr;  // [kKernelCount]
    struct Ev {
        int kid;
        hipEvent_t a, b;
    };
    std::vector<Ev> pending_ev;
    std::vector<hipEvent_t> ev_pool;
    // the asynchronous move end's side stream (UTTT_SEED_STREAM=1): k_archive runs there behind
    // k_finalize (ev_fin) and the next move end waits for it (ev_seed, join_seed)
    hipStream_t seed_stream = nullptr;
    hipEvent_t ev_fin = nullptr, ev_seed = nullptr;
    bool seed_inflight = false;
    double ms[kKernelCount] = {};
    int64_t launches[kKernelCount] = {};
    std::vector<void *> allocs;
};

namespace {

int dev_alloc(uttt_engine *e, void **p, size_t bytes) {
    if (bytes == 0) bytes = 16;
    hipError_t r = hipMalloc(p, bytes);
    if (r != hipSuccess) {
        set_error("hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(r));
        return UTTT_ERR_HIP;
    }
    e->allocs.push_back(*p);
    e->bytes += (int64_t)bytes;
    return UTTT_OK;
}

template <typename T>
int alloc_n(uttt_engine *e, T **p, size_t n) {
    return dev_alloc(e, reinterpret_cast<void **>(p), n * sizeof(T));
}

hipEvent_t get_event(uttt_engine *e) {
    if (!e->ev_pool.empty()) {
        hipEvent_t ev = e->ev_pool.back();
        e->ev_pool.pop_back();
        return ev;
    }
    hipEvent_t ev;
    // timing-only events: no system-scope fence when recorded (the default one flushes caches at
    // every record; with ~8 timed launches per round that was visible in the tree-only rounds). No
    // host reads data through these events (the counts and counters are system-scope stores).
    if (hipEventCreateWithFlags(&ev, hipEventDisableSystemFence) != hipSuccess) return nullptr;
    return ev;
}

struct TimedLaunch {
    uttt_engine *e;
    int kid;
    hipEvent_t a = nullptr, b = nullptr;
    TimedLaunch(uttt_engine *e_, int kid_) : e(e_), kid(kid_) {
        e->launches[kid]++;
        if (e->timing) {
            a = get_event(e);
            b = get_event(e);
            if (a) (void)hipEventRecord(a, e->stream);
        }
    }
    ~TimedLaunch() {
        if (e->timing && a && b) {
            (void)hipEventRecord(b, e->stream);
            e->pending_ev.push_back({kid, a, b});
        }
    }
};

// One kernel launch whose time the engine's telemetry keeps (round 5): with timing on, the start and
// stop events are the dispatch's own (hipExtLaunchKernelGGL records them when the kernel starts and
// completes, as rocprofv3's kernel trace measures it), not marker packets around the launch: a marker
// pair added ~10 us per launch to the tree kernels (tree-only k_select 27.9 us under rocprofv3 against
// 38.0 us between markers, k_apply 8.5 against 18.7; gpurun_out/t5a, profiles/r5/summary_tree_only.md).
template <typename K, typename... Args>
void timed_launch(uttt_engine *e, int kid, K kernel, dim3 grid, dim3 block, Args... args) {
    e->launches[kid]++;
    if (e->timing) {
        hipEvent_t a = get_event(e), b = get_event(e);
        if (a && b) {
            hipExtLaunchKernelGGL(kernel, grid, block, 0, e->stream, a, b, 0, args...);
            e->pending_ev.push_back({kid, a, b});
            return;
        }
        if (a) e->ev_pool.push_back(a);
        if (b) e->ev_pool.push_back(b);
    }
    hipLaunchKernelGGL(kernel, grid, block, 0, e->stream, args...);
}

// Fold finished event pairs into the totals (pairs whose end has not been reached yet, e.g.
// behind the asynchronous rounds, stay pending).
void drain_events(uttt_engine *e) {
    size_t keep = 0;
    for (auto &ev : e->pending_ev) {
        if (hipEventQuery(ev.b) == hipErrorNotReady) {
            e->pending_ev[keep++] = ev;
            continue;
        }
        float ms = 0.0f;
        if (hipEventElapsedTime(&ms, ev.a, ev.b) == hipSuccess) e->ms[ev.kid] += ms;
        e->ev_pool.push_back(ev.a);
        e->ev_pool.push_back(ev.b);
    }
    e->pending_ev.resize(keep);
}

unsigned long long *bytes_ptr(uttt_engine *e, int kid) { return e->timing ? e->d_bytes + (size_t)kid * kRow : nullptr; }

int check_launch() {
    hipError_t r = hipGetLastError();
    if (r != hipSuccess) {
        set_error("kernel launch failed: %s", hipGetErrorString(r));
        return UTTT_ERR_HIP;
    }
    return UTTT_OK;
}

int grid_waves(int waves) { return (waves + kWavesPerBlock - 1) / kWavesPerBlock; }

int ensure_scratch(uttt_engine *e, int64_t rows) {
    if (rows <= e->scratch_rows) return UTTT_OK;
    int64_t n = e->scratch_rows ? e->scratch_rows : 1024;
    while (n < rows) n *= 2;
    if (e->d_pol_scratch) {
        (void)hipFree(e->d_pol_scratch);
        (void)hipFree(e->d_val_scratch);
        (void)hipFree(e->d_rowbase);
    }
    HIP_TRY(hipMalloc((void **)&e->d_pol_scratch, (size_t)n * 81 * sizeof(float)));
    HIP_TRY(hipMalloc((void **)&e->d_val_scratch, (size_t)n * sizeof(float)));
    HIP_TRY(hipMalloc((void **)&e->d_rowbase, (size_t)std::max<int64_t>(n, e->max_trees) * sizeof(int32_t)));
    e->scratch_rows = n;
    return UTTT_OK;
}

}  // namespace

namespace uttt {
// For the evaluator kernels (nn_kernels.hip): the pending leaves of the current round.
// After uttt_search_select_async the count is on the device only: *n = -1, *n_dev points at
// it and *max_n bounds it (launch grids sized for max_n, kernels exit past *n_dev).
int engine_pending_view(uttt_engine_t *e, const uttt_state_t **leaf, const int32_t **tree_of, int32_t *n,
                        const int32_t **n_dev, int32_t *max_n, hipStream_t *stream) {
    if (!e) return UTTT_ERR_ARG;
    if (e->phase != 2 && e->phase != 3) {
        set_error("no pending leaves (call uttt_search_select first)");
        return UTTT_ERR_ORDER;
    }
    *leaf = e->tr.leaf;
    *tree_of = e->tr.tree_of;
    *n = e->phase == 2 ? e->n_pending : -1;
    *n_dev = e->phase == 3 ? e->tr.count : nullptr;
    *max_n = e->tr.n_trees;
    *stream = e->stream;
    return UTTT_OK;
}
}  // namespace uttt

extern "C" {

const char *uttt_version(void) { return "uttt-mi355x 0.1 (gfx950)"; }

int uttt_engine_create(int32_t device, int32_t max_trees, int32_t max_sims, uttt_engine_t **out) {
    if (!out || max_trees <= 0 || max_trees >= (1 << 21) || max_sims <= 0 || max_sims > kMaxSimsRec) {
        // (k_scan packs its three per-round counts into 21-bit fields)
        set_error("uttt_engine_create: bad arguments (max_trees=%d of at most 2097151, max_sims=%d of at most %d)",
                  max_trees, max_sims, kMaxSimsRec);
        return UTTT_ERR_ARG;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        set_error("no HIP device visible");
        return UTTT_ERR_NODEVICE;
    }
    if (device < 0 && hipGetDevice(&device) != hipSuccess) device = 0;
    if (device < 0 || device >= ndev) {
        set_error("device %d out of range (%d visible)", device, ndev);
        return UTTT_ERR_NODEVICE;
    }
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        set_error("device %d is %s; this engine is built for gfx950 (MI355X)", device, prop.gcnArchName);
        return UTTT_ERR_NODEVICE;
    }
    HIP_TRY(hipSetDevice(device));
    uttt_engine *e = new uttt_engine();
    e->device = device;
    e->max_trees = max_trees;
    e->max_sims = max_sims;
    e->cap = 82 + 81ll * max_sims;  // root + 81 children + 81 per consumed simulation (exact bound)
    int rc = UTTT_OK;
    auto fail = [&](int code) {
        uttt_engine_destroy(e);
        return code;
    };
    if (hipStreamCreateWithFlags(&e->own_stream, hipStreamNonBlocking) != hipSuccess) return fail(UTTT_ERR_HIP);
    e->stream = e->own_stream;
    const size_t nodes = (size_t)max_trees * (size_t)e->cap;
    e->pool.cap = e->cap;
    if ((rc = alloc_n(e, &e->pool.rec, nodes))) return fail(rc);
    if ((rc = alloc_n(e, &e->tr.ctl, max_trees)) || (rc = alloc_n(e, &e->tr.root, max_trees)) ||
        (rc = alloc_n(e, &e->tr.leaf, max_trees)) || (rc = alloc_n(e, &e->tr.rec, max_trees)) ||
        (rc = alloc_n(e, &e->tr.path, (size_t)max_trees * kMaxDepth)) ||
        (rc = alloc_n(e, &e->tr.path_rec, (size_t)max_trees * kMaxDepth)) || (rc = alloc_n(e, &e->tr.pending, max_trees)) ||
        (rc = alloc_n(e, &e->tr.tree_of, max_trees)) || (rc = alloc_n(e, &e->tr.depth_of, max_trees)) ||
        (rc = alloc_n(e, &e->tr.slot_of, max_trees)) || (rc = alloc_n(e, &e->tr.count, 4)) ||
        (rc = alloc_n(e, &e->d_scores, (size_t)max_trees * 81)) || (rc = alloc_n(e, &e->d_visits, (size_t)max_trees * 81)) ||
        (rc = alloc_n(e, &e->d_nlegal, max_trees)) || (rc = alloc_n(e, &e->d_bytes, kKernelCount * kRow)) ||
        (rc = alloc_n(e, &e->d_cache_ctr, 4 * kRow)) ||
        (rc = alloc_n(e, &e->d_r1ctl, (size_t)kR1Partial + (size_t)grid_waves(max_trees))))
        return fail(rc);
    if ((rc = alloc_n(e, &e->d_err, 1))) return fail(rc);
    if (hipHostMalloc((void **)&e->h_move, sizeof(int64_t) * 5, hipHostMallocCoherent) != hipSuccess) {
        set_error("hipHostMalloc failed");
        return fail(UTTT_ERR_HIP);
    }
    if (hipHostMalloc((void **)&e->h_ring, sizeof(int32_t) * 4 * kCountRing, hipHostMallocCoherent) != hipSuccess) {
        set_error("hipHostMalloc failed");
        return fail(UTTT_ERR_HIP);
    }
    memset(e->h_ring, 0, sizeof(int32_t) * 4 * kCountRing);
    if (hipHostMalloc((void **)&e->h_leaf, sizeof(HostLeaf), hipHostMallocCoherent) != hipSuccess) {
        set_error("hipHostMalloc failed");
        return fail(UTTT_ERR_HIP);
    }
    memset(e->h_leaf, 0, sizeof(HostLeaf));
    if (hipHostMalloc((void **)&e->h_count, sizeof(int32_t) * 4, hipHostMallocDefault) != hipSuccess) {
        set_error("hipHostMalloc failed");
        return fail(UTTT_ERR_HIP);
    }
    if (hipMemsetAsync(e->tr.ctl, 0, sizeof(TreeCtl) * max_trees, e->stream) != hipSuccess ||
        hipMemsetAsync(e->d_bytes, 0, sizeof(unsigned long long) * kKernelCount * kRow, e->stream) != hipSuccess ||
        hipMemsetAsync(e->d_cache_ctr, 0, sizeof(unsigned long long) * 4 * kRow, e->stream) != hipSuccess ||
        hipMemsetAsync(e->d_r1ctl, 0, sizeof(uint32_t) * ((size_t)kR1Partial + (size_t)grid_waves(max_trees)),
                       e->stream) != hipSuccess ||
        hipStreamSynchronize(e->stream) != hipSuccess) {
        set_error("engine init memset failed");
        return fail(UTTT_ERR_HIP);
    }
    e->tr.n_trees = 0;
    *out = e;
    return UTTT_OK;
}

static int search1_stop(uttt_engine *e);
int uttt_engine_destroy(uttt_engine_t *e) {
    if (!e) return UTTT_OK;
    (void)hipSetDevice(e->device);
    (void)search1_stop(e);  // a resident one-tree search wave exits first
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    drain_events(e);
    if (e->seed_stream) (void)hipStreamSynchronize(e->seed_stream);
    if (e->ev_fin) (void)hipEventDestroy(e->ev_fin);
    if (e->ev_seed) (void)hipEventDestroy(e->ev_seed);
    if (e->seed_stream) (void)hipStreamDestroy(e->seed_stream);
    for (hipEvent_t ev : e->ev_pool) (void)hipEventDestroy(ev);
    for (void *p : e->allocs) (void)hipFree(p);
    if (e->d_pol_scratch) (void)hipFree(e->d_pol_scratch);
    if (e->d_val_scratch) (void)hipFree(e->d_val_scratch);
    if (e->d_rowbase) (void)hipFree(e->d_rowbase);
    if (e->cache_owner) {
        if (e->cache.flag) (void)hipFree(e->cache.flag);
        if (e->cache.rec) (void)hipFree(e->cache.rec);
    }
    if (e->h_count) (void)hipHostFree(e->h_count);
    if (e->h_ring) (void)hipHostFree(e->h_ring);
    if (e->h_part) (void)hipHostFree(e->h_part);
    if (e->h_leaf) (void)hipHostFree(e->h_leaf);
    if (e->h_eval) (void)hipHostFree(e->h_eval);
    if (e->h_s1) (void)hipHostFree(e->h_s1);
    if (e->h_move) (void)hipHostFree(e->h_move);
    if (e->own_stream) (void)hipStreamDestroy(e->own_stream);
    delete e;
    return UTTT_OK;
}

int uttt_engine_own_stream(uttt_engine_t *e, void **stream) {
    if (!e || !stream) return UTTT_ERR_ARG;
    *stream = (void *)e->own_stream;
    return UTTT_OK;
}

int uttt_engine_set_stream(uttt_engine_t *e, void *stream) {
    if (!e) return UTTT_ERR_ARG;
    // NULL is the null (legacy default) stream — what torch.cuda.current_stream()
    // is unless the caller made one; the engine's own stream is non-blocking and
    // would not be ordered against it.
    e->stream = (hipStream_t)stream;
    return UTTT_OK;
}

int64_t uttt_engine_device_bytes(const uttt_engine_t *e) { return e ? e->bytes : 0; }

static int search1_stop(uttt_engine *e);
static int search_begin_common(uttt_engine *e, int32_t n_trees, int32_t sims, int32_t batch) {
    if (int rc0 = search1_stop(e)) return rc0;  // a resident one-tree search left unfinished
    e->dev_apply_staged = false;  // a staged round of a search that was never ended is dropped with it
    e->host_apply_rows = 0;       // (and a staged one-tree evaluation)
    if (n_trees <= 0 || n_trees > e->max_trees) {
        set_error("n_trees %d out of range 1..%d", n_trees, e->max_trees);
        return UTTT_ERR_ARG;
    }
    if (sims <= 0 || sims > e->max_sims) {
        set_error("evaluate_count %d out of range 1..%d (engine max_sims)", sims, e->max_sims);
        return UTTT_ERR_ARG;
    }
    e->tr.n_trees = n_trees;
    e->tr.sims = sims;
    // uttt_mcts.cpp:127: a flush happens once the queue holds batch_size entries,
    // so batch_size <= 1 flushes every queued leaf alone.
    e->tr.batch = batch < 1 ? 1 : batch;
    // the select budget changes how a move's simulations are spread over launches, never which
    // simulations run or in what order per tree (results are the same for any value >= 1)
    const char *bv = getenv("UTTT_SELECT_BUDGET");
    const int b = bv ? atoi(bv) : 0;
    e->tr.budget = b >= 1 && b <= 4096 ? b : kSelectBudget;
    e->phase = 1;
    e->n_pending = 0;
    return UTTT_OK;
}

int uttt_search_begin(uttt_engine_t *e, const uttt_state_t *roots, int32_t n_trees, int32_t sims, int32_t batch) {
    return uttt_search_begin_mode(e, roots, n_trees, sims, batch, UTTT_SEMANTICS_CPP);
}

int uttt_search_begin_mode(uttt_engine_t *e, const uttt_state_t *roots, int32_t n_trees, int32_t sims, int32_t batch,
                           int32_t semantics) {
    if (!e || !roots || (semantics != UTTT_SEMANTICS_CPP && semantics != UTTT_SEMANTICS_PY)) {
        set_error("uttt_search_begin_mode: bad arguments (semantics 0 = cpp, 1 = py)");
        return UTTT_ERR_ARG;
    }
    HIP_TRY(hipSetDevice(e->device));
    e->host_apply_rows = 0;  // a staged evaluation of the previous search is dropped with it
    e->dev_apply_staged = false;
    int rc = search_begin_common(e, n_trees, sims, batch);
    if (rc) return rc;
    e->tr.py = semantics == UTTT_SEMANTICS_PY ? 1 : 0;
    e->selfplay = false;
    HIP_TRY(hipMemcpyAsync(e->tr.leaf, roots, sizeof(uttt_state_t) * n_trees, hipMemcpyHostToDevice, e->stream));
    hipLaunchKernelGGL(k_begin, dim3(grid_waves(n_trees)), dim3(kBlock), 0, e->stream, e->pool, e->tr,
                       (const char *)e->tr.leaf, (int)sizeof(uttt_state_t), (const int32_t *)nullptr,
                       (unsigned long long *)nullptr);
    return check_launch();
}

static int flush_host_apply(uttt_engine *e);

int uttt_search_select(uttt_engine_t *e, float *nn_input, int32_t *n_pending) {
    if (!e || !n_pending) return UTTT_ERR_ARG;
    if (e->phase != 1) {
        set_error("uttt_search_select: call uttt_search_begin (or apply the previous round) first");
        return UTTT_ERR_ORDER;
    }
    HIP_TRY(hipSetDevice(e->device));
    if (int rc0 = flush_host_apply(e)) return rc0;
    int rc = 0, n = 0;
    // trees stopped by the select budget resume in the next launch; when no tree has a
    // leaf but some were stopped, select again (every launch completes >= 1 simulation
    // of each stopped tree, so this ends)
    for (;;) {
        timed_launch(e, kKSelect, e->tr.py ? k_select<true> : k_select<false>, dim3(grid_waves(e->tr.n_trees)),
                     dim3(kBlock), e->pool, e->tr, e->cache, e->timing ? e->d_bytes : nullptr);
        if ((rc = check_launch())) return rc;
        timed_launch(e, kKScan, k_scan, dim3(1), dim3(1024), e->tr, e->timing ? e->d_bytes : nullptr,
                     (int32_t *)nullptr, (int32_t)0);
        if ((rc = check_launch())) return rc;
        HIP_TRY(hipMemcpyAsync(e->h_count, e->tr.count, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, e->stream));
        HIP_TRY(hipStreamSynchronize(e->stream));
        drain_events(e);
        n = e->h_count[0];
        if (n > 0 || e->h_count[1] == 0) break;
    }
    if (n > 0 && nn_input) {
        const int total = n * 243;
        timed_launch(e, kKEncode, k_encode, dim3((total + 255) / 256), dim3(256), e->tr, nn_input, n);
    }
    if ((rc = check_launch())) return rc;
    e->n_pending = n;
    e->phase = n > 0 ? 2 : 1;
    *n_pending = n;
    return UTTT_OK;
}

static int select_async_impl(uttt_engine_t *e, int32_t *host_count, int32_t tag = 0);
int uttt_search_select_async(uttt_engine_t *e) { return select_async_impl(e, nullptr); }

int uttt_search_select_async_to(uttt_engine_t *e, int32_t ring_slot) {
    if (!e || ring_slot < 0 || ring_slot >= kCountRing) {
        set_error("uttt_search_select_async_to: ring slot must be in 0..%d", kCountRing - 1);
        return UTTT_ERR_ARG;
    }
    return select_async_impl(e, e->h_ring + 4 * ring_slot);
}

int uttt_search_select_async_tag(uttt_engine_t *e, int32_t ring_slot, int32_t tag) {
    if (!e || ring_slot < 0 || ring_slot >= kCountRing) {
        set_error("uttt_search_select_async_tag: ring slot must be in 0..%d", kCountRing - 1);
        return UTTT_ERR_ARG;
    }
    return select_async_impl(e, e->h_ring + 4 * ring_slot, tag);
}

int uttt_search_count_ring(uttt_engine_t *e, const int32_t **ring, int32_t *n_slots) {
    if (!e || !ring || !n_slots) return UTTT_ERR_ARG;
    *ring = e->h_ring;
    *n_slots = kCountRing;
    return UTTT_OK;
}

static int select_async_impl(uttt_engine_t *e, int32_t *host_count, int32_t tag) {
    if (!e) return UTTT_ERR_ARG;
    if (e->phase != 1) {
        set_error("uttt_search_select_async: call uttt_search_begin (or apply the previous round) first");
        return UTTT_ERR_ORDER;
    }
    HIP_TRY(hipSetDevice(e->device));
    if (int rc0 = flush_host_apply(e)) return rc0;
    int rc = 0;
    timed_launch(e, kKSelect, e->tr.py ? k_select<true> : k_select<false>, dim3(grid_waves(e->tr.n_trees)),
                 dim3(kBlock), e->pool, e->tr, e->cache, e->timing ? e->d_bytes : nullptr);
    if ((rc = check_launch())) return rc;
    timed_launch(e, kKScan, k_scan, dim3(1), dim3(1024), e->tr, e->timing ? e->d_bytes : nullptr, host_count, tag);
    if ((rc = check_launch())) return rc;
    e->n_pending = -1;
    e->phase = 3;
    return UTTT_OK;
}

int uttt_search_count_copy(uttt_engine_t *e, int32_t *dst) {
    if (!e || !dst) return UTTT_ERR_ARG;
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipMemcpyAsync(dst, e->tr.count, 3 * sizeof(int32_t), hipMemcpyDeviceToHost, e->stream));
    return UTTT_OK;
}

int uttt_search_count_ptr(uttt_engine_t *e, const int32_t **count) {
    if (!e || !count) return UTTT_ERR_ARG;
    *count = e->tr.count;
    return UTTT_OK;
}

int uttt_search_pending(uttt_engine_t *e, uttt_state_t *states, int32_t *copies) {
    if (!e) return UTTT_ERR_ARG;
    if (e->phase != 2) {
        set_error("uttt_search_pending: no pending leaves (call uttt_search_select)");
        return UTTT_ERR_ORDER;
    }
    HIP_TRY(hipSetDevice(e->device));
    const int n = e->n_pending;
    std::vector<int32_t> tree_of(n);
    HIP_TRY(hipMemcpyAsync(tree_of.data(), e->tr.tree_of, sizeof(int32_t) * n, hipMemcpyDeviceToHost, e->stream));
    std::vector<uttt_state_t> leaf(e->tr.n_trees);
    std::vector<LeafRec> rec(e->tr.n_trees);
    HIP_TRY(hipMemcpyAsync(leaf.data(), e->tr.leaf, sizeof(uttt_state_t) * e->tr.n_trees, hipMemcpyDeviceToHost,
                           e->stream));
    HIP_TRY(hipMemcpyAsync(rec.data(), e->tr.rec, sizeof(LeafRec) * e->tr.n_trees, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    for (int i = 0; i < n; ++i) {
        if (states) states[i] = leaf[tree_of[i]];
        if (copies) copies[i] = rec[tree_of[i]].k;
    }
    return UTTT_OK;
}

// Wait for a tag the device stores into fine-grained host memory (k_scan): spin, no stream sync.
static int wait_host_tag(uttt_engine *e, const int32_t *tag_word, int32_t tag) {
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 1;; ++it) {
        if (__atomic_load_n(tag_word, __ATOMIC_ACQUIRE) == tag) return UTTT_OK;
        if ((it & 1023u) == 0u) {
            const hipError_t q = hipStreamQuery(e->stream);
            if (q != hipSuccess && q != hipErrorNotReady) {
                set_error("engine stream failed: %s", hipGetErrorString(q));
                return UTTT_ERR_HIP;
            }
            if (q == hipSuccess && __atomic_load_n(tag_word, __ATOMIC_ACQUIRE) != tag) {
                set_error("engine: the stream drained without storing the round's tag");
                return UTTT_ERR_HIP;
            }
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) {
                set_error("engine: round result not stored within 60 s");
                return UTTT_ERR_HIP;
            }
        }
        __builtin_ia32_pause();
    }
}

// The staged evaluation's k_apply arguments (pinned host memory; rows 1: one row for the leaf's k copies,
// rows k: one per copy, applied in order, the evaluation cache bypassed as in uttt_search_apply).
struct HostApplyArgs {
    const float *policy, *value;
    const int32_t *rowbase;
    int per_copy;
    EvalCache cache;
};
static HostApplyArgs host_apply_args(uttt_engine *e) {
    HostApplyArgs a;
    a.policy = e->h_eval;
    a.value = e->h_eval + e->h_eval_rows * 96;
    a.rowbase = reinterpret_cast<const int32_t *>(e->h_eval + e->h_eval_rows * 97);
    a.per_copy = e->host_apply_rows > 1 ? 1 : 0;
    a.cache = a.per_copy ? EvalCache{} : e->cache;
    return a;
}

// A round's evaluation staged by uttt_round_hash_async that no k_round has applied yet, applied now (by
// every call that reads, selects in or restarts the trees, uttt_search_select_host included)
static int flush_dev_apply(uttt_engine *e) {
    if (!e->dev_apply_staged) return UTTT_OK;
    e->dev_apply_staged = false;
    if (e->dev_apply_by_tree) {  // a one-dispatch round's rows, by tree
        e->dev_apply_by_tree = false;
        timed_launch(e, kKApply, k_apply_tree, dim3(grid_waves(e->tr.n_trees)), dim3(kBlock), e->pool, e->tr, e->cache,
                     e->dev_apply_policy, e->dev_apply_value, bytes_ptr(e, kKApply));
        return check_launch();
    }
    // the phase-3 form of uttt_search_apply: every tree's wave, the count read on the device
    timed_launch(e, kKApply, k_apply, dim3(grid_waves(e->tr.n_trees)), dim3(kBlock), e->pool, e->tr, e->cache,
                 e->dev_apply_policy, (int64_t)81, e->dev_apply_value, (int64_t)1, (const int32_t *)nullptr, 0,
                 bytes_ptr(e, kKApply));
    return check_launch();
}

static int flush_host_apply(uttt_engine *e) {
    if (int rc = flush_dev_apply(e)) return rc;
    if (!e->host_apply_rows) return UTTT_OK;
    const HostApplyArgs a = host_apply_args(e);
    e->host_apply_rows = 0;
    timed_launch(e, kKApply, k_apply, dim3(grid_waves(1)), dim3(kBlock), e->pool, e->tr, a.cache, a.policy,
                 (int64_t)96, a.value, (int64_t)1, a.rowbase, a.per_copy, bytes_ptr(e, kKApply));
    return check_launch();
}

// ---- the resident one-tree search (k_search1) ----
static float *s1_policy(uttt_engine *e) { return reinterpret_cast<float *>(e->h_s1 + 1); }
static float *s1_value(uttt_engine *e) { return s1_policy(e) + (size_t)e->s1_cap * 96; }

// a resident wave left by an unfinished search exits (its exit word) before anything else runs on the stream
static int search1_stop(uttt_engine *e) {
    if (!e->s1_alive) return UTTT_OK;
    __atomic_store_n(&e->h_s1->cmd_exit, 1, __ATOMIC_SEQ_CST);
    e->s1_alive = false;
    HIP_TRY(hipStreamSynchronize(e->stream));
    return UTTT_OK;
}

static int search1_launch(uttt_engine *e, int32_t resume) {
    hipLaunchKernelGGL(e->tr.py ? k_search1<true> : k_search1<false>, dim3(1), dim3(kWave), 0, e->stream, e->pool, e->tr,
                       e->cache, e->s1_root, e->s1_temperature, e->h_s1, (const float *)s1_policy(e),
                       (const float *)s1_value(e), e->s1_seq, resume);
    e->s1_alive = true;
    return check_launch();
}

int uttt_search1_begin(uttt_engine_t *e, const uttt_state_t *root, int32_t sims, int32_t batch, int32_t semantics,
                       float temperature) {
    if (!e || !root || (semantics != UTTT_SEMANTICS_CPP && semantics != UTTT_SEMANTICS_PY)) {
        set_error("uttt_search1_begin: bad arguments (semantics 0 = cpp, 1 = py)");
        return UTTT_ERR_ARG;
    }
    HIP_TRY(hipSetDevice(e->device));
    if (int rc0 = search1_stop(e)) return rc0;
    int rc = search_begin_common(e, 1, sims, batch);
    if (rc) return rc;
    e->tr.py = semantics == UTTT_SEMANTICS_PY ? 1 : 0;
    e->selfplay = false;
    const int32_t need = e->tr.batch > 16 ? e->tr.batch : 16;  // rows per flush: 1 or k <= batch
    if (need > e->s1_cap) {
        if (e->h_s1) (void)hipHostFree(e->h_s1);  // no wave is resident (search1_stop)
        e->h_s1 = nullptr;
        e->s1_cap = 0;
        const size_t bytes = sizeof(Search1Host) + (size_t)need * 97 * sizeof(float) + 16;
        if (hipHostMalloc((void **)&e->h_s1, bytes, hipHostMallocCoherent) != hipSuccess) {
            set_error("hipHostMalloc failed");
            return UTTT_ERR_HIP;
        }
        memset((void *)e->h_s1, 0, bytes);
        e->s1_cap = need;
    }
    Search1Host *h = e->h_s1;
    h->tag = 0;
    h->gone = 0;
    h->cmd = 0;
    h->cmd_exit = 0;
    h->count = 0;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    e->s1_root = *root;
    e->s1_temperature = temperature;
    e->s1_seq = 0;
    e->phase = 1;
    e->n_pending = 0;
    return search1_launch(e, 0);
}

int uttt_search1_next(uttt_engine_t *e, uttt_state_t *leaf, int32_t *copies, int32_t *n_pending) {
    if (!e || !leaf || !copies || !n_pending) return UTTT_ERR_ARG;
    if (e->phase != 1 || !e->h_s1 || !e->s1_alive) {
        set_error("uttt_search1_next: call uttt_search1_begin (or apply the previous leaf) first");
        return UTTT_ERR_ORDER;
    }
    const int32_t want = e->s1_seq + 1;
    Search1Host *h = e->h_s1;
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 1;; ++it) {
        if (__atomic_load_n(&h->tag, __ATOMIC_ACQUIRE) == want) break;
        // the stream is queried only for a wait past 20 ms (the wave's 100 ms timeout, a failed stream): a
        // query goes through the runtime's locks (uttt_rounds_hash_move)
        if ((it & 255u) == 0u && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) {
            const hipError_t q = hipStreamQuery(e->stream);
            if (q != hipSuccess && q != hipErrorNotReady) {
                set_error("engine stream failed: %s", hipGetErrorString(q));
                return UTTT_ERR_HIP;
            }
            if (q == hipSuccess && __atomic_load_n(&h->tag, __ATOMIC_ACQUIRE) != want) {
                // the wave timed out waiting for the previous command (the host took over 100 ms): resume it,
                // the command it did not see applied first
                if (__atomic_load_n(&h->gone, __ATOMIC_ACQUIRE) != e->s1_seq || e->s1_seq == 0) {
                    set_error("engine: the resident search left without storing its result");
                    return UTTT_ERR_HIP;
                }
                h->gone = 0;
                __atomic_thread_fence(__ATOMIC_SEQ_CST);
                if (int rc0 = search1_launch(e, 1)) return rc0;
            }
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) {
                set_error("engine: one-tree search result not stored within 60 s");
                return UTTT_ERR_HIP;
            }
        }
        __builtin_ia32_pause();
    }
    e->s1_seq = want;
    const int n = __atomic_load_n(&h->count, __ATOMIC_ACQUIRE);
    if (n > 0) {
        memcpy(leaf, const_cast<const uttt_state_t *>(&h->leaf), sizeof(uttt_state_t));
        *copies = h->k;
        e->n_pending = 1;
        e->phase = 2;
    } else {
        e->s1_alive = false;  // the wave ends after the search's end
        e->n_pending = 0;
        e->phase = 1;
        const uint32_t st = (uint32_t)__atomic_load_n(&h->status, __ATOMIC_ACQUIRE);
        if (st & kErrMask) {
            set_error("tree 0 failed (status 0x%x: %s)", st, tree_error_text(st));
            return tree_error_code(st);
        }
    }
    *n_pending = n;
    return UTTT_OK;
}

int uttt_search1_apply(uttt_engine_t *e, const float *policy, int64_t pld, const float *value, int32_t rows) {
    if (!e || !policy || !value || pld < 81 || rows < 1) {
        set_error("uttt_search1_apply: bad arguments (policy stride must be >= 81, rows >= 1)");
        return UTTT_ERR_ARG;
    }
    if (e->phase != 2 || !e->s1_alive) {
        set_error("uttt_search1_apply: no pending leaf (call uttt_search1_next)");
        return UTTT_ERR_ORDER;
    }
    Search1Host *h = e->h_s1;
    const int32_t k = h->k;
    if ((rows != 1 && rows != k) || rows > e->s1_cap) {
        set_error("uttt_search1_apply: %d results for a leaf queued %d times (pass 1 or %d)", rows, k, k);
        return UTTT_ERR_ARG;
    }
    float *hp = s1_policy(e), *hv = s1_value(e);
    for (int32_t r = 0; r < rows; ++r) {
        memcpy(hp + (size_t)r * 96, policy + (size_t)r * pld, 81 * sizeof(float));
        hv[r] = value[r];
    }
    // the rows before the command the wave polls (x86 keeps stores in order; the fence keeps the compiler's)
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    __atomic_store_n(&h->cmd, (uint64_t)(uint32_t)rows << 32 | (uint32_t)e->s1_seq, __ATOMIC_RELEASE);
    e->phase = 1;
    e->n_pending = 0;
    return UTTT_OK;
}

int uttt_search1_scores(uttt_engine_t *e, float *scores, int32_t *n_legal) {
    if (!e || !scores || !n_legal) return UTTT_ERR_ARG;
    if (!e->h_s1 || e->s1_alive || e->phase != 1) {
        set_error("uttt_search1_scores: the search has not ended (uttt_search1_next returns no leaf at its end)");
        return UTTT_ERR_ORDER;
    }
    const Search1Host *h = e->h_s1;
    const int L = h->n_legal;
    for (int i = 0; i < 81; ++i) scores[i] = i < L ? h->scores[i] : 0.0f;
    *n_legal = L;
    return UTTT_OK;
}

int uttt_search1_time_split(uttt_engine_t *e, int32_t *ticks3) {
    if (!e || !ticks3 || !e->h_s1) return UTTT_ERR_ARG;
    const Search1Host *h = e->h_s1;
    ticks3[0] = __atomic_load_n(&h->t_select, __ATOMIC_ACQUIRE);
    ticks3[1] = __atomic_load_n(&h->t_apply, __ATOMIC_ACQUIRE);
    ticks3[2] = __atomic_load_n(&h->t_wait, __ATOMIC_ACQUIRE);
    return UTTT_OK;
}

int uttt_search_select_host(uttt_engine_t *e, uttt_state_t *leaf, int32_t *copies, int32_t *n_pending) {
    if (!e || !leaf || !copies || !n_pending) return UTTT_ERR_ARG;
    if (e->tr.n_trees != 1) {
        set_error("uttt_search_select_host: one-tree searches only (uttt_search_begin with n_trees = 1)");
        return UTTT_ERR_ARG;
    }
    if (e->phase != 1) {
        set_error("uttt_search_select_host: call uttt_search_begin (or apply the previous round) first");
        return UTTT_ERR_ORDER;
    }
    HIP_TRY(hipSetDevice(e->device));
    // a round staged by uttt_round_hash_async on this one-tree search is applied first (k_flush1 applies only
    // host-staged evaluations)
    if (int rc0 = flush_dev_apply(e)) return rc0;
    int rc = 0, n = 0;
    for (;;) {  // the select budget may stop the tree before it queues a leaf: select again (as uttt_search_select)
        const int32_t tag = ++e->leaf_tag;
        const int do_apply = e->host_apply_rows ? 1 : 0;
        HostApplyArgs a = host_apply_args(e);
        e->host_apply_rows = 0;
        e->launches[kKApply] += do_apply;
        timed_launch(e, kKSelect, e->tr.py ? k_flush1<true> : k_flush1<false>, dim3(1), dim3(kWave), e->pool, e->tr,
                     e->cache, a.cache, a.policy, (int64_t)96, a.value, (int64_t)1, a.rowbase, a.per_copy, do_apply,
                     e->timing ? e->d_bytes : nullptr, e->h_leaf, tag);
        if ((rc = check_launch())) return rc;
        if ((rc = wait_host_tag(e, &e->h_leaf->tag, tag))) return rc;
        n = __atomic_load_n(&e->h_leaf->count, __ATOMIC_ACQUIRE);
        if (e->timing) drain_events(e);
        if (n > 0 || __atomic_load_n(&e->h_leaf->stopped, __ATOMIC_ACQUIRE) == 0) break;
    }
    if (n > 0) {
        memcpy(leaf, const_cast<const uttt_state_t *>(&e->h_leaf->state), sizeof(uttt_state_t));
        *copies = e->h_leaf->k;
    }
    *n_pending = n;
    e->n_pending = n;
    e->phase = n > 0 ? 2 : 1;
    return UTTT_OK;
}

int uttt_search_apply_host(uttt_engine_t *e, const float *policy, int64_t pld, const float *value, int32_t rows) {
    if (!e || !policy || !value || pld < 81 || rows < 1) {
        set_error("uttt_search_apply_host: bad arguments (policy stride must be >= 81, rows >= 1)");
        return UTTT_ERR_ARG;
    }
    if (e->phase != 2 || e->n_pending != 1 || e->tr.n_trees != 1) {
        set_error("uttt_search_apply_host: no pending leaf of a one-tree search (call uttt_search_select_host)");
        return UTTT_ERR_ORDER;
    }
    const int32_t k = e->h_leaf->k;
    if (rows != 1 && rows != k) {
        set_error("uttt_search_apply_host: %d results for a leaf queued %d times (pass 1 or %d)", rows, k, k);
        return UTTT_ERR_ARG;
    }
    HIP_TRY(hipSetDevice(e->device));
    if (rows > e->h_eval_rows) {
        // grown between rounds only: the k_flush1 that last read the buffer completed before it stored the
        // tag the host has seen
        if (e->h_eval) (void)hipHostFree(e->h_eval);
        e->h_eval = nullptr;
        int64_t cap = e->h_eval_rows ? e->h_eval_rows : 16;
        while (cap < rows) cap *= 2;
        if (hipHostMalloc((void **)&e->h_eval, (size_t)cap * 97 * sizeof(float) + 16, hipHostMallocCoherent) != hipSuccess) {
            e->h_eval_rows = 0;
            set_error("hipHostMalloc failed");
            return UTTT_ERR_HIP;
        }
        e->h_eval_rows = cap;
        reinterpret_cast<int32_t *>(e->h_eval + cap * 97)[0] = 0;  // the per-copy row base of slot 0
    }
    float *hp = e->h_eval, *hv = e->h_eval + e->h_eval_rows * 96;
    for (int32_t r = 0; r < rows; ++r) {
        memcpy(hp + (size_t)r * 96, policy + (size_t)r * pld, 81 * sizeof(float));
        hv[r] = value[r];
    }
    __atomic_thread_fence(__ATOMIC_SEQ_CST);  // before the launch that reads them
    e->host_apply_rows = rows;  // applied by the next k_flush1 (or flush_host_apply)
    e->phase = 1;
    e->n_pending = 0;
    return UTTT_OK;
}

int uttt_search_apply(uttt_engine_t *e, const float *policy, int64_t pld, const float *value, int64_t vld,
                      int32_t per_copy, int32_t on_device) {
    if (!e || !policy || !value || pld < 81 || vld < 1) {
        set_error("uttt_search_apply: bad arguments (policy stride must be >= 81)");
        return UTTT_ERR_ARG;
    }
    if (e->phase != 2 && e->phase != 3) {
        set_error("uttt_search_apply: no pending leaves (call uttt_search_select)");
        return UTTT_ERR_ORDER;
    }
    if (e->phase == 3 && (per_copy || !on_device)) {
        set_error("uttt_search_apply: after uttt_search_select_async the results must be on the device, one per leaf");
        return UTTT_ERR_ORDER;
    }
    if (per_copy && e->tr.py) {
        set_error("uttt_search_apply: per_copy is the cpp call pattern; py semantics take one result per leaf");
        return UTTT_ERR_ARG;
    }
    HIP_TRY(hipSetDevice(e->device));
    // phase 3: the count is on the device; k_apply reads it (tr.count[0]) and the grid covers every tree
    const int n = e->phase == 3 ? e->tr.n_trees : e->n_pending;
    const int32_t *rowbase = nullptr;
    int64_t rows = n;
    if (per_copy) {
        // rows are grouped per slot: slot i's k_i copies start at sum_{j<i} k_j
        std::vector<int32_t> k(n);
        int rc = uttt_search_pending(e, nullptr, k.data());
        if (rc) return rc;
        std::vector<int32_t> rb(n);
        int64_t acc = 0;
        for (int i = 0; i < n; ++i) {
            rb[i] = (int32_t)acc;
            acc += k[i];
        }
        rows = acc;
        if ((rc = ensure_scratch(e, rows))) return rc;
        HIP_TRY(hipMemcpyAsync(e->d_rowbase, rb.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, e->stream));
        rowbase = e->d_rowbase;
    }
    const float *dp = policy, *dv = value;
    int64_t dpld = pld, dvld = vld;
    if (!on_device) {
        int rc = ensure_scratch(e, rows);
        if (rc) return rc;
        HIP_TRY(hipMemcpy2DAsync(e->d_pol_scratch, 81 * sizeof(float), policy, (size_t)pld * sizeof(float),
                                 81 * sizeof(float), (size_t)rows, hipMemcpyHostToDevice, e->stream));
        HIP_TRY(hipMemcpy2DAsync(e->d_val_scratch, sizeof(float), value, (size_t)vld * sizeof(float), sizeof(float),
                                 (size_t)rows, hipMemcpyHostToDevice, e->stream));
        dp = e->d_pol_scratch;
        dv = e->d_val_scratch;
        dpld = 81;
        dvld = 1;
    }
    {
        EvalCache c = per_copy ? EvalCache{} : e->cache;  // the reference call pattern bypasses the cache
        timed_launch(e, kKApply, k_apply, dim3(grid_waves(n)), dim3(kBlock), e->pool, e->tr, c, dp, dpld, dv, dvld,
                     rowbase, per_copy ? 1 : 0, bytes_ptr(e, kKApply));
    }
    int rc = check_launch();
    if (rc) return rc;
    if (!on_device) HIP_TRY(hipStreamSynchronize(e->stream));  // host buffers may be freed on return
    e->phase = 1;
    e->n_pending = 0;
    return UTTT_OK;
}

int uttt_eval_hash(uttt_engine_t *e, const float *nn_input, int32_t n, float *policy, float *value) {
    if (!e || !nn_input || !policy || !value || n < 0) return UTTT_ERR_ARG;
    if (n == 0) return UTTT_OK;
    HIP_TRY(hipSetDevice(e->device));
    timed_launch(e, kKHash, k_hash_eval, dim3(grid_waves(n)), dim3(kBlock), nn_input, n, policy, value);
    return check_launch();
}

int uttt_eval_hash_dev(uttt_engine_t *e, float *policy, float *value) {
    if (!e || !policy || !value) return UTTT_ERR_ARG;
    HIP_TRY(hipSetDevice(e->device));
    timed_launch(e, kKHash, k_hash_leaves, dim3(grid_waves(e->tr.n_trees)), dim3(kBlock), e->tr, policy, value);
    return check_launch();
}

// the first round after a begin (nothing staged): the plain select, then this round's evaluation staged
static int select_async_then_stage(uttt_engine *e, int32_t ring_slot, int32_t tag, float *policy, float *value) {
    int rc = select_async_impl(e, e->h_ring + 4 * ring_slot, tag);
    if (rc) return rc;
    if ((rc = uttt_eval_hash_dev(e, policy, value))) return rc;
    e->dev_apply_policy = policy;
    e->dev_apply_value = value;
    e->dev_apply_staged = true;
    e->dev_apply_by_tree = false;
    e->phase = 1;
    e->n_pending = 0;
    return UTTT_OK;
}

int uttt_round_hash_async(uttt_engine_t *e, int32_t ring_slot, int32_t tag, float *policy, float *value);

int uttt_rounds_hash_async(uttt_engine_t *e, int32_t ring_slot, int32_t tag, float *policy, float *value,
                           int32_t n_rounds) {
    if (!e || n_rounds < 1 || n_rounds > kCountRing) {
        set_error("uttt_rounds_hash_async: n_rounds must be in 1..%d", kCountRing);
        return UTTT_ERR_ARG;
    }
    for (int32_t i = 0; i < n_rounds; ++i)
        if (int rc = uttt_round_hash_async(e, (ring_slot + i) % kCountRing, tag + i, policy, value)) return rc;
    return UTTT_OK;
}

static int round_hash_async_impl(uttt_engine *e, int32_t ring_slot, int32_t tag, float *policy, float *value,
                                 uint32_t *part_host, uint32_t *part_dev, const uint32_t *part_prev, int nb_prev,
                                 int stats_parity = 0);

static bool one_dispatch_rounds() {  // k_round1 (UTTT_ROUND_DISPATCHES=3 / UTTT_FUSED_ROUNDS=0: the round-5 forms)
    static const bool one = [] {
        const char *f = getenv("UTTT_FUSED_ROUNDS"), *d = getenv("UTTT_ROUND_DISPATCHES");
        return !(f && f[0] == '0') && !(d && d[0] == '3');
    }();
    return one;
}

int uttt_rounds_hash_move(uttt_engine_t *e, int32_t ring_slot, int32_t tag, float *policy, float *value, int32_t depth,
                          int32_t *n_rounds, int64_t *n_leaves, int32_t *n_with_leaves) {
    if (!e || !n_rounds || !n_leaves || !n_with_leaves || depth < 1 || depth >= kCountRing || ring_slot < 0 ||
        ring_slot >= kCountRing) {
        set_error("uttt_rounds_hash_move: bad arguments (depth in 1..%d, ring slot in 0..%d)", kCountRing - 1,
                  kCountRing - 1);
        return UTTT_ERR_ARG;
    }
    // per-block count words (k_round1's part_host form: no last-block publish; UTTT_ROUND_PARTS=0 keeps the ring
    // slot's counts); with kernel timing, each round folds the previous round's select statistics (rows by
    // round parity) at its start
    static const bool parts_env = [] {
        const char *v = getenv("UTTT_ROUND_PARTS");
        return !(v && v[0] == '0');
    }();
    const bool parts = parts_env && one_dispatch_rounds();
    const int nb = grid_waves(e->tr.n_trees);
    if (parts && !e->h_part) {
        const int cap = grid_waves(e->max_trees);
        if (hipHostMalloc((void **)&e->h_part, sizeof(uint32_t) * (size_t)kCountRing * cap, hipHostMallocCoherent) !=
            hipSuccess) {
            set_error("hipHostMalloc failed");
            return UTTT_ERR_HIP;
        }
        memset(e->h_part, 0xFF, sizeof(uint32_t) * (size_t)kCountRing * cap);  // no word valid (n0 field 31)
        if (int rc = alloc_n(e, &e->d_part, (size_t)2 * cap)) return rc;
        e->part_cap = cap;
    }
    const int cap = e->part_cap;
    int32_t enq = 0, head = 0, with_leaves = 0;
    int64_t leaves = 0;
    auto tag_of = [tag](int32_t i) { return (int32_t)(((uint32_t)tag + (uint32_t)i) & 0x7FFFFFFFu); };
    auto push = [&]() -> int {
        const int slot = (ring_slot + enq) % kCountRing;
        const int rc = parts ? round_hash_async_impl(e, slot, tag_of(enq), policy, value, e->h_part + (size_t)slot * cap,
                                                     e->d_part + (size_t)(enq & 1) * cap,
                                                     enq ? e->d_part + (size_t)((enq - 1) & 1) * cap : nullptr, nb,
                                                     (e->round_parity++) & 1)
                             : uttt_round_hash_async(e, slot, tag_of(enq), policy, value);
        if (rc == UTTT_OK) ++enq;
        return rc;
    };
    auto finish = [&](int rc) {
        *n_rounds = enq;
        *n_leaves = leaves;
        *n_with_leaves = with_leaves;
        return rc;
    };
    // the spin's failure checks: the stream is queried only for a wait past 20 ms (a failed or finished
    // stream): a query while the rounds run goes through the runtime's locks and cost tree-only self-play 7%
    // when made every ~40 us (round 6)
    auto still_waiting = [&](const std::chrono::steady_clock::time_point &t0, unsigned it, auto &&ready) -> int {
        if ((it & 1023u) == 0u && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) {
            const hipError_t q = hipStreamQuery(e->stream);
            if (q != hipSuccess && q != hipErrorNotReady) {
                set_error("engine stream failed: %s", hipGetErrorString(q));
                return UTTT_ERR_HIP;
            }
            if (q == hipSuccess && !ready()) {
                set_error("engine: a hash round ended without storing its counts");
                return UTTT_ERR_HIP;
            }
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) {
                set_error("engine: a hash round's counts not stored within 60 s");
                return UTTT_ERR_HIP;
            }
        }
        __builtin_ia32_pause();
        return UTTT_OK;
    };
    for (int32_t i = 0; i < depth; ++i)
        if (int rc = push()) return finish(rc);
    for (;;) {
        const int slot = (ring_slot + head) % kCountRing;
        const int32_t want = tag_of(head);
        const auto t0 = std::chrono::steady_clock::now();
        int32_t n = 0, left = 0;
        if (parts) {  // every block's word carries this round's tag: sum them
            const uint32_t *pw = e->h_part + (size_t)slot * cap;
            const uint32_t want17 = (uint32_t)want & kPartTagMask;
            auto word_ok = [&](uint32_t w) { return (w >> kPartTagShift) == want17 && (w & 0x1Fu) <= 16u; };
            int i = 0;
            auto all_ready = [&] {
                for (int j = 0; j < nb; ++j)
                    if (!word_ok(__atomic_load_n(pw + j, __ATOMIC_ACQUIRE))) return false;
                return true;
            };
            for (unsigned it = 1; i < nb; ++it) {
                while (i < nb && word_ok(__atomic_load_n(pw + i, __ATOMIC_ACQUIRE))) ++i;
                if (i < nb)
                    if (int rc = still_waiting(t0, it, all_ready)) return finish(rc);
            }
            for (int j = 0; j < nb; ++j) {
                const uint32_t w = __atomic_load_n(pw + j, __ATOMIC_ACQUIRE);
                n += (int32_t)(w & 0x1Fu);
                left += (int32_t)((w >> 10) & 0x1Fu);
            }
        } else {
            const int32_t *w = e->h_ring + 4 * slot;
            auto ready = [&] { return __atomic_load_n(w + 3, __ATOMIC_ACQUIRE) == want; };
            for (unsigned it = 1; !ready(); ++it)
                if (int rc = still_waiting(t0, it, ready)) return finish(rc);
            n = __atomic_load_n(w + 0, __ATOMIC_ACQUIRE);
            left = __atomic_load_n(w + 2, __ATOMIC_ACQUIRE);
        }
        leaves += n;
        with_leaves += n > 0 ? 1 : 0;
        ++head;
        if (left <= 0) {  // the move's last round: the ones behind it are empty
            // a round enqueued behind it applied its leaves and queued none, so the evaluation staged by the
            // last enqueued round is empty: the move end need not flush it (one k_apply_tree launch less)
            if (enq > head) e->dev_apply_staged = false;
            return finish(UTTT_OK);
        }
        if (int rc = push()) return finish(rc);
    }
}

int uttt_round_hash_async(uttt_engine_t *e, int32_t ring_slot, int32_t tag, float *policy, float *value) {
    return round_hash_async_impl(e, ring_slot, tag, policy, value, nullptr, nullptr, nullptr, 0);
}

// part_host != nullptr (uttt_rounds_hash_move only, with the one-dispatch rounds): the round's counts go to
// per-block words instead of the ring slot (k_round1's part_host form)
static int round_hash_async_impl(uttt_engine *e, int32_t ring_slot, int32_t tag, float *policy, float *value,
                                 uint32_t *part_host, uint32_t *part_dev, const uint32_t *part_prev, int nb_prev,
                                 int stats_parity) {
    if (!e || !policy || !value || ring_slot < 0 || ring_slot >= kCountRing) {
        set_error("uttt_round_hash_async: bad arguments (ring slot must be in 0..%d)", kCountRing - 1);
        return UTTT_ERR_ARG;
    }
    static const bool fuse = [] {
        const char *v = getenv("UTTT_FUSED_ROUNDS");
        return !(v && v[0] == '0');
    }();
    // round 6: the whole round in one dispatch (k_round1; UTTT_ROUND_DISPATCHES=3 keeps k_round + k_scan +
    // k_hash_leaves)
    if (one_dispatch_rounds()) {
        if (e->phase != 1) {
            set_error("uttt_round_hash_async: call uttt_search_begin (or apply the previous round) first");
            return UTTT_ERR_ORDER;
        }
        HIP_TRY(hipSetDevice(e->device));
        if (e->host_apply_rows) {  // (a one-tree host evaluation cannot be staged beside a round's)
            if (int rc0 = flush_host_apply(e)) return rc0;
        }
        if (e->dev_apply_staged && !e->dev_apply_by_tree)  // staged by a slot-order round: apply it first
            if (int rc0 = flush_dev_apply(e)) return rc0;
        const int apply = e->dev_apply_staged ? 1 : 0;
        timed_launch(e, kKSelect, e->tr.py ? k_round1<true> : k_round1<false>, dim3(grid_waves(e->tr.n_trees)),
                     dim3(kBlock), e->pool, e->tr, e->cache, e->dev_apply_policy, e->dev_apply_value, policy, value, apply,
                     e->timing ? e->d_bytes : nullptr, e->h_ring + 4 * ring_slot, tag, e->d_r1ctl, part_host, part_dev,
                     part_prev, nb_prev, stats_parity);
        if (int rc0 = check_launch()) return rc0;
        e->dev_apply_policy = policy;
        e->dev_apply_value = value;
        e->dev_apply_staged = true;
        e->dev_apply_by_tree = true;
        e->phase = 1;
        e->n_pending = 0;
        return UTTT_OK;
    }
    if (!fuse) {
        int rc = select_async_impl(e, e->h_ring + 4 * ring_slot, tag);
        if (rc) return rc;
        if ((rc = uttt_eval_hash_dev(e, policy, value))) return rc;
        return uttt_search_apply(e, policy, 81, value, 1, 0, 1);
    }
    // the previous round's apply and this round's select as one k_round launch; this round's apply is staged
    if (!e->dev_apply_staged) return select_async_then_stage(e, ring_slot, tag, policy, value);
    if (e->phase != 1) {
        set_error("uttt_round_hash_async: call uttt_search_begin (or apply the previous round) first");
        return UTTT_ERR_ORDER;
    }
    HIP_TRY(hipSetDevice(e->device));
    if (e->host_apply_rows) {  // (a one-tree host evaluation cannot be staged beside a round's)
        set_error("uttt_round_hash_async: a host-staged evaluation is pending");
        return UTTT_ERR_ORDER;
    }
    e->dev_apply_staged = false;
    int rc = 0;
    timed_launch(e, kKSelect, e->tr.py ? k_round<true> : k_round<false>, dim3(grid_waves(e->tr.n_trees)),
                 dim3(kBlock), e->pool, e->tr, e->cache, e->dev_apply_policy, (int64_t)81, e->dev_apply_value,
                 (int64_t)1, e->timing ? e->d_bytes : nullptr);
    if ((rc = check_launch())) return rc;
    timed_launch(e, kKScan, k_scan, dim3(1), dim3(1024), e->tr, e->timing ? e->d_bytes : nullptr,
                 e->h_ring + 4 * ring_slot, tag);
    if ((rc = check_launch())) return rc;
    e->n_pending = -1;
    e->phase = 3;
    if ((rc = uttt_eval_hash_dev(e, policy, value))) return rc;
    e->dev_apply_policy = policy;
    e->dev_apply_value = value;
    e->dev_apply_staged = true;
    e->dev_apply_by_tree = false;
    e->phase = 1;
    e->n_pending = 0;
    return UTTT_OK;
}

static int check_tree_errors(uttt_engine *e) {
    std::vector<TreeCtl> ctl(e->tr.n_trees);
    HIP_TRY(hipMemcpyAsync(ctl.data(), e->tr.ctl, sizeof(TreeCtl) * e->tr.n_trees, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    for (int t = 0; t < e->tr.n_trees; ++t) {
        if (ctl[t].status & kErrMask) {
            set_error("tree %d failed (status 0x%x: %s)", t, ctl[t].status, tree_error_text((uint32_t)ctl[t].status));
            return tree_error_code((uint32_t)ctl[t].status);
        }
    }
    return UTTT_OK;
}

int uttt_search_root_visits(uttt_engine_t *e, int32_t *visits, int32_t *n_legal) {
    if (!e) return UTTT_ERR_ARG;
    HIP_TRY(hipSetDevice(e->device));
    if (int rc0 = flush_host_apply(e)) return rc0;
    int rc = check_tree_errors(e);
    if (rc) return rc;
    const int n = e->tr.n_trees;
    hipLaunchKernelGGL(k_root_visits, dim3((n * 81 + 255) / 256), dim3(256), 0, e->stream, e->pool, e->tr, e->d_visits,
                       e->d_nlegal);
    if ((rc = check_launch())) return rc;
    if (visits)
        HIP_TRY(hipMemcpyAsync(visits, e->d_visits, sizeof(int32_t) * 81 * n, hipMemcpyDeviceToHost, e->stream));
    if (n_legal) HIP_TRY(hipMemcpyAsync(n_legal, e->d_nlegal, sizeof(int32_t) * n, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return UTTT_OK;
}

int uttt_search_scores(uttt_engine_t *e, float temperature, float *scores, int32_t *n_legal) {
    if (!e) return UTTT_ERR_ARG;
    HIP_TRY(hipSetDevice(e->device));
    if (int rc0 = flush_host_apply(e)) return rc0;
    int rc = check_tree_errors(e);
    if (rc) return rc;
    const int n = e->tr.n_trees;
    hipLaunchKernelGGL(k_root_scores, dim3((n + 255) / 256), dim3(256), 0, e->stream, e->pool, e->tr, temperature,
                       e->d_scores, e->d_nlegal);
    if ((rc = check_launch())) return rc;
    if (scores) HIP_TRY(hipMemcpyAsync(scores, e->d_scores, sizeof(float) * 81 * n, hipMemcpyDeviceToHost, e->stream));
    if (n_legal) HIP_TRY(hipMemcpyAsync(n_legal, e->d_nlegal, sizeof(int32_t) * n, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return UTTT_OK;
}

// ----------------------------------------------------------- self-play API --
// The engine's stream waits for a key seeding still running on the side stream (every self-play call that
// reads or writes keys, slots or the work list on the stream joins first)
static int join_seed(uttt_engine *e) {
    if (!e->seed_inflight) return UTTT_OK;
    HIP_TRY(hipStreamWaitEvent(e->stream, e->ev_seed, 0));
    e->seed_inflight = false;
    return UTTT_OK;
}

int uttt_selfplay_begin(uttt_engine_t *e, int64_t game_begin, int64_t game_end, uint32_t seed_base, float temperature,
                        int32_t sims, int32_t batch, int64_t arena_plies) {
    if (!e || game_end < game_begin || game_begin < 0 || arena_plies <= 0) {
        set_error("uttt_selfplay_begin: bad arguments");
        return UTTT_ERR_ARG;
    }
    HIP_TRY(hipSetDevice(e->device));
    if (int rc_join = join_seed(e)) return rc_join;
    const int slots = e->max_trees;
    int rc = search_begin_common(e, slots, sims, batch);
    e->tr.py = 0;  // self-play is the cpp/uttt_mcts.cpp path
    if (rc) return rc;
    e->phase = 0;  // move_begin first
    SelfPlay &sp = e->sp;
    if (!sp.slot) {
        if ((rc = alloc_n(e, &sp.slot, slots)) || (rc = alloc_n(e, &sp.mt_key, (size_t)slots * 624)) ||
            (rc = alloc_n(e, &sp.mt_pos, slots)) || (rc = alloc_n(e, &sp.ply_state, (size_t)slots * kMaxPlies)) ||
            (rc = alloc_n(e, &sp.ply_policy, (size_t)slots * kMaxPlies * 81)) ||
            (rc = alloc_n(e, &sp.ply_action, (size_t)slots * kMaxPlies)) || (rc = alloc_n(e, &sp.ctr, 4)) ||
            (rc = alloc_n(e, &sp.live, slots)) || (rc = alloc_n(e, &sp.work, (size_t)slots + 1)))
            return rc;
    }
    // every archived game has >= 1 ply, so the arena bounds the game table too
    const int64_t games = std::min<int64_t>(game_end - game_begin, arena_plies);
    if (sp.arena_cap < arena_plies) {
        if (sp.ar_state) {
            (void)hipFree(sp.ar_state);
            (void)hipFree(sp.ar_policy);
            (void)hipFree(sp.ar_action);
            (void)hipFree(sp.ar_value);
        }
        HIP_TRY(hipMalloc((void **)&sp.ar_state, sizeof(uttt_state_t) * arena_plies));
        HIP_TRY(hipMalloc((void **)&sp.ar_policy, sizeof(double) * 81 * arena_plies));
        HIP_TRY(hipMalloc((void **)&sp.ar_action, arena_plies));
        HIP_TRY(hipMalloc((void **)&sp.ar_value, arena_plies));
        sp.arena_cap = arena_plies;
    }
    if (sp.games_cap < games || !sp.games) {
        if (sp.games) (void)hipFree(sp.games);
        HIP_TRY(hipMalloc((void **)&sp.games, sizeof(GameEntry) * std::max<int64_t>(games, 1)));
        sp.games_cap = std::max<int64_t>(games, 1);
    }
    sp.game_end = game_end;
    sp.seed_base = seed_base;
    sp.temperature = temperature;
    sp.slots = slots;
    // every slot starts free; k_finalize hands out games [game_begin, ...)
    HIP_TRY(hipMemsetAsync(sp.slot, 0, sizeof(Slot) * slots, e->stream));
    int64_t ctr[4] = {game_begin, 0, 0, 0};
    HIP_TRY(hipMemcpyAsync(sp.ctr, ctr, sizeof(ctr), hipMemcpyHostToDevice, e->stream));
    hipLaunchKernelGGL(k_finalize, dim3(1), dim3(1024), 0, e->stream, sp, (const int32_t *)nullptr,
                       (const TreeCtl *)nullptr, (unsigned long long *)nullptr, (int64_t *)nullptr);
    hipLaunchKernelGGL(k_archive, dim3(archive_grid(slots)), dim3(256), 0, e->stream, sp, (const unsigned long long *)nullptr, 1);
    if ((rc = check_launch())) return rc;
    HIP_TRY(hipMemcpyAsync(e->h_move, sp.ctr, sizeof(int64_t) * 4, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    e->h_move[4] = -1;
    e->selfplay = true;
    e->sp_arena_used = 0;
    e->moves = 0;
    return uttt_engine_cache_clear(e);  // a new run may use a new model
}

int uttt_selfplay_move_begin(uttt_engine_t *e, int32_t *n_live) {
    if (!e || !e->selfplay) {
        set_error("uttt_selfplay_move_begin: call uttt_selfplay_begin first");
        return UTTT_ERR_ORDER;
    }
    HIP_TRY(hipSetDevice(e->device));
    if (int rc_join = join_seed(e)) return rc_join;
    const int slots = e->sp.slots;
    e->tr.n_trees = slots;
    if (e->cache.flag && e->cache_clear_every > 0 && e->moves > 0 && e->moves % e->cache_clear_every == 0) {
        int rc0 = uttt_engine_cache_clear(e);
        if (rc0) return rc0;
    }
    e->dev_apply_staged = false;  // (a move that was never ended)
    e->host_apply_rows = 0;       // (a one-tree evaluation staged by a search on this engine, never applied)
    e->moves++;
    // roots = the slots' current positions (Slot.state is the first member)
    std::vector<int32_t> live(slots);
    HIP_TRY(hipMemcpyAsync(live.data(), e->sp.live, sizeof(int32_t) * slots, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    int nl = 0;
    for (int v : live) nl += v != 0;
    if (n_live) *n_live = nl;
    // roots: the slots' states, read in place (Slot.state is the first member)
    hipLaunchKernelGGL(k_begin, dim3(grid_waves(slots)), dim3(kBlock), 0, e->stream, e->pool, e->tr,
                       (const char *)e->sp.slot, (int)sizeof(Slot), (const int32_t *)e->sp.live, e->d_err);
    int rc = check_launch();
    if (rc) return rc;
    e->phase = 1;
    e->n_pending = 0;
    return UTTT_OK;
}

int uttt_selfplay_move_end(uttt_engine_t *e, int64_t *n_finished) {
    if (!e || !e->selfplay) {
        set_error("uttt_selfplay_move_end: call uttt_selfplay_begin first");
        return UTTT_ERR_ORDER;
    }
    if (e->phase == 2 || e->phase == 3) {
        set_error("uttt_selfplay_move_end: pending leaves were not applied");
        return UTTT_ERR_ORDER;
    }
    HIP_TRY(hipSetDevice(e->device));
    if (int rc_join = join_seed(e)) return rc_join;
    if (int rc0 = flush_host_apply(e)) return rc0;  // a staged round's evaluation (uttt_round_hash_async)
    int rc = check_tree_errors(e);
    if (rc) return rc;
    const int slots = e->sp.slots;
    {
        TimedLaunch tl(e, kKMoveEnd);
        const unsigned long long *no_err = nullptr;
        hipLaunchKernelGGL(k_move_end, dim3((slots + kWavesPerBlock - 1) / kWavesPerBlock), dim3(kBlock), 0, e->stream,
                           e->pool, e->sp, (const int32_t *)nullptr);
        hipLaunchKernelGGL(k_finalize, dim3(1), dim3(1024), 0, e->stream, e->sp, (const int32_t *)nullptr,
                           (const TreeCtl *)nullptr, (unsigned long long *)nullptr, (int64_t *)nullptr);
        hipLaunchKernelGGL(k_archive, dim3(archive_grid(slots)), dim3(256), 0, e->stream, e->sp, no_err, 1);
    }
    if ((rc = check_launch())) return rc;
    int64_t ctr[4];
    HIP_TRY(hipMemcpyAsync(ctr, e->sp.ctr, sizeof(ctr), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    drain_events(e);
    if (ctr[2] > e->sp.arena_cap) {
        set_error("self-play record arena full (%lld plies > %lld)", (long long)ctr[2], (long long)e->sp.arena_cap);
        return UTTT_ERR_CAPACITY;
    }
    e->sp_arena_used = ctr[2];
    if (n_finished) *n_finished = ctr[1];
    e->phase = 0;
    return UTTT_OK;
}

int uttt_selfplay_move_begin_async(uttt_engine_t *e) {
    if (!e || !e->selfplay) {
        set_error("uttt_selfplay_move_begin_async: call uttt_selfplay_begin first");
        return UTTT_ERR_ORDER;
    }
    if (e->phase != 0) {
        set_error("uttt_selfplay_move_begin_async: the previous move was not ended");
        return UTTT_ERR_ORDER;
    }
    if (e->cache.flag && e->cache_clear_every > 0) {
        set_error("uttt_selfplay_move_begin_async: periodic cache clears need the blocking move_begin");
        return UTTT_ERR_ORDER;
    }
    HIP_TRY(hipSetDevice(e->device));
    const int slots = e->sp.slots;
    e->dev_apply_staged = false;  // (a move that was never ended)
    e->host_apply_rows = 0;       // (a one-tree evaluation staged by a search on this engine, never applied)
    e->tr.n_trees = slots;
    e->moves++;
    hipLaunchKernelGGL(k_begin, dim3(grid_waves(slots)), dim3(kBlock), 0, e->stream, e->pool, e->tr,
                       (const char *)e->sp.slot, (int)sizeof(Slot), (const int32_t *)e->sp.live, e->d_err);
    int rc = check_launch();
    if (rc) return rc;
    e->phase = 1;
    e->n_pending = 0;
    return UTTT_OK;
}

int uttt_selfplay_move_end_async(uttt_engine_t *e) {
    if (!e || !e->selfplay) {
        set_error("uttt_selfplay_move_end_async: call uttt_selfplay_begin first");
        return UTTT_ERR_ORDER;
    }
    if (e->phase != 1) {
        set_error("uttt_selfplay_move_end_async: no move in progress, or pending leaves were not applied");
        return UTTT_ERR_ORDER;
    }
    HIP_TRY(hipSetDevice(e->device));
    if (int rc0 = flush_host_apply(e)) return rc0;  // a staged round's evaluation (uttt_round_hash_async)
    if (int rc0 = join_seed(e)) return rc0;         // the previous move end's key seeding
    const int slots = e->sp.slots;
    {  // d_err and the failure flag were reset by this move's k_begin
        TimedLaunch tl(e, kKMoveEnd);
        // a failed tree leaves the whole move unended (the failure flag, set where a tree's status gets an
        // error bit; k_finalize then puts the first failed tree into *d_err, which k_archive checks), so the
        // engine is in the state the blocking move end refuses in
        const int32_t *fail = e->tr.count + 3;
        const unsigned long long *err = e->d_err;
        hipLaunchKernelGGL(k_move_end, dim3((slots + kWavesPerBlock - 1) / kWavesPerBlock), dim3(kBlock), 0, e->stream,
                           e->pool, e->sp, fail);
        hipLaunchKernelGGL(k_finalize, dim3(1), dim3(1024), 0, e->stream, e->sp, fail, (const TreeCtl *)e->tr.ctl,
                           e->d_err, e->h_move);
        // UTTT_SEED_STREAM=1: k_archive (the finished games' copy to the arena, the refilled slots' keys) runs
        // on a side stream, overlapping the next move's rounds, which need neither; the next move end and every
        // reader of the arena or the keys join it (round 6, measured in DESIGN §7)
        static const bool side = [] {
            const char *v = getenv("UTTT_SEED_STREAM");
            return v && v[0] == '1';
        }();
        if (side) {
            if (!e->seed_stream) {
                HIP_TRY(hipStreamCreateWithFlags(&e->seed_stream, hipStreamNonBlocking));
                HIP_TRY(hipEventCreateWithFlags(&e->ev_fin, hipEventDisableTiming | hipEventDisableSystemFence));
                HIP_TRY(hipEventCreateWithFlags(&e->ev_seed, hipEventDisableTiming | hipEventDisableSystemFence));
            }
            HIP_TRY(hipEventRecord(e->ev_fin, e->stream));
            HIP_TRY(hipStreamWaitEvent(e->seed_stream, e->ev_fin, 0));
            hipLaunchKernelGGL(k_archive, dim3(archive_grid(slots)), dim3(256), 0, e->seed_stream, e->sp, err, 1);
            HIP_TRY(hipEventRecord(e->ev_seed, e->seed_stream));
            e->seed_inflight = true;
        } else {
            hipLaunchKernelGGL(k_archive, dim3(archive_grid(slots)), dim3(256), 0, e->stream, e->sp, err, 1);
        }
    }
    int rc = check_launch();
    if (rc) return rc;  // k_finalize stored the counters and the failure word into h_move
    e->phase = 0;
    return UTTT_OK;
}

int uttt_selfplay_move_result(uttt_engine_t *e, int64_t *n_finished, int32_t *n_live_next) {
    if (!e || !e->selfplay) return UTTT_ERR_ORDER;
    const unsigned long long err = (unsigned long long)e->h_move[4];
    if (err != ~0ull) {
        const uint32_t st = (uint32_t)err, t = (uint32_t)(err >> 32);
        set_error("tree %u failed (status 0x%x: %s)", t, st, tree_error_text(st));
        return tree_error_code(st);
    }
    if (e->h_move[2] > e->sp.arena_cap) {
        set_error("self-play record arena full (%lld plies > %lld)", (long long)e->h_move[2],
                  (long long)e->sp.arena_cap);
        return UTTT_ERR_CAPACITY;
    }
    e->sp_arena_used = e->h_move[2];
    drain_events(e);
    if (n_finished) *n_finished = e->h_move[1];
    if (n_live_next) *n_live_next = (int32_t)e->h_move[3];
    return UTTT_OK;
}

int uttt_selfplay_games(uttt_engine_t *e, int64_t *game_ids, int64_t *offsets, int32_t *lengths, int64_t max_games,
                        int64_t *n_games) {
    if (!e || !e->selfplay) return UTTT_ERR_ORDER;
    HIP_TRY(hipSetDevice(e->device));
    if (int rc_join = join_seed(e)) return rc_join;
    int64_t ctr[4];
    HIP_TRY(hipMemcpyAsync(ctr, e->sp.ctr, sizeof(ctr), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    const int64_t n = std::min<int64_t>(ctr[1], e->sp.games_cap);
    std::vector<GameEntry> g((size_t)n);
    if (n) HIP_TRY(hipMemcpy(g.data(), e->sp.games, sizeof(GameEntry) * n, hipMemcpyDeviceToHost));
    std::sort(g.begin(), g.end(), [](const GameEntry &a, const GameEntry &b) { return a.game < b.game; });
    const int64_t m = std::min<int64_t>(n, max_games);
    for (int64_t i = 0; i < m; ++i) {
        if (game_ids) game_ids[i] = g[i].game;
        if (offsets) offsets[i] = g[i].offset;
        if (lengths) lengths[i] = (int32_t)g[i].length;
    }
    if (n_games) *n_games = n;
    return UTTT_OK;
}

int uttt_selfplay_plies(uttt_engine_t *e, uttt_state_t *states, double *policies, int8_t *actions, int8_t *values,
                        float *inputs_hwc, int64_t max_plies, int64_t *n_plies) {
    if (!e || !e->selfplay) return UTTT_ERR_ORDER;
    HIP_TRY(hipSetDevice(e->device));
    if (int rc_join = join_seed(e)) return rc_join;
    const int64_t n = std::min<int64_t>(e->sp_arena_used, max_plies);
    if (n_plies) *n_plies = e->sp_arena_used;
    if (n <= 0) return UTTT_OK;
    if (states) HIP_TRY(hipMemcpy(states, e->sp.ar_state, sizeof(uttt_state_t) * n, hipMemcpyDeviceToHost));
    if (policies) HIP_TRY(hipMemcpy(policies, e->sp.ar_policy, sizeof(double) * 81 * n, hipMemcpyDeviceToHost));
    if (actions) HIP_TRY(hipMemcpy(actions, e->sp.ar_action, n, hipMemcpyDeviceToHost));
    if (values) HIP_TRY(hipMemcpy(values, e->sp.ar_value, n, hipMemcpyDeviceToHost));
    if (inputs_hwc) {
        float *d = nullptr;
        HIP_TRY(hipMalloc((void **)&d, sizeof(float) * 243 * n));
        hipLaunchKernelGGL(k_hwc, dim3((unsigned)((n * 81 + 255) / 256)), dim3(256), 0, e->stream, e->sp.ar_state, n, d);
        hipError_t r = hipGetLastError();
        if (r == hipSuccess) r = hipStreamSynchronize(e->stream);
        if (r == hipSuccess) r = hipMemcpy(inputs_hwc, d, sizeof(float) * 243 * n, hipMemcpyDeviceToHost);
        (void)hipFree(d);
        if (r != hipSuccess) {
            set_error("history tensor expansion failed: %s", hipGetErrorString(r));
            return UTTT_ERR_HIP;
        }
    }
    return UTTT_OK;
}

int uttt_selfplay_get_rng(uttt_engine_t *e, int32_t slot, uint32_t key[624], int32_t *pos) {
    if (!e || !e->selfplay || slot < 0 || slot >= e->sp.slots || !key || !pos) return UTTT_ERR_ARG;
    HIP_TRY(hipSetDevice(e->device));
    if (int rc_join = join_seed(e)) return rc_join;
    HIP_TRY(hipMemcpyAsync(key, e->sp.mt_key + (size_t)slot * 624, sizeof(uint32_t) * 624, hipMemcpyDeviceToHost,
                           e->stream));
    HIP_TRY(hipMemcpyAsync(pos, e->sp.mt_pos + slot, sizeof(int32_t), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return UTTT_OK;
}

int uttt_selfplay_set_rng(uttt_engine_t *e, int32_t slot, const uint32_t key[624], int32_t pos) {
    if (!e || !e->selfplay || slot < 0 || slot >= e->sp.slots || !key || pos < 0 || pos > 624) return UTTT_ERR_ARG;
    HIP_TRY(hipSetDevice(e->device));
    if (int rc_join = join_seed(e)) return rc_join;
    HIP_TRY(hipMemcpyAsync(e->sp.mt_key + (size_t)slot * 624, key, sizeof(uint32_t) * 624, hipMemcpyHostToDevice,
                           e->stream));
    HIP_TRY(hipMemcpyAsync(e->sp.mt_pos + slot, &pos, sizeof(int32_t), hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return UTTT_OK;
}

// ------------------------------------------------------- evaluation cache --
int uttt_engine_set_cache(uttt_engine_t *e, int32_t log2_capacity, int32_t clear_every_moves) {
    if (!e || log2_capacity < 0 || log2_capacity > 26 || clear_every_moves < 0) {
        set_error("uttt_engine_set_cache: log2_capacity must be 0 (off) .. 26");
        return UTTT_ERR_ARG;
    }
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipStreamSynchronize(e->stream));
    if (e->cache.flag && e->cache_owner) {
        (void)hipFree(e->cache.flag);
        (void)hipFree(e->cache.rec);
        e->bytes -= (int64_t)((sizeof(uint32_t) + kRecBytes) << e->cache_log2);
    }
    e->cache = EvalCache{};
    e->cache_owner = true;
    e->cache_log2 = log2_capacity;
    e->cache_clear_every = clear_every_moves;
    if (log2_capacity == 0) return UTTT_OK;
    const size_t cap = (size_t)1 << log2_capacity;
    HIP_TRY(hipMalloc((void **)&e->cache.flag, sizeof(uint32_t) * cap));
    HIP_TRY(hipMalloc((void **)&e->cache.rec, (size_t)kRecBytes * cap));
    e->bytes += (int64_t)((sizeof(uint32_t) + kRecBytes) * cap);
    e->cache.mask = (uint32_t)(cap - 1);
    e->cache.ctr = e->d_cache_ctr;
    return uttt_engine_cache_clear(e);
}

int uttt_engine_share_cache(uttt_engine_t *e, uttt_engine_t *owner) {
    if (!e || !owner || e == owner || !owner->cache_owner || e->device != owner->device) {
        set_error("uttt_engine_share_cache: need a distinct owner engine (with its own table) on the same device");
        return UTTT_ERR_ARG;
    }
    int rc = uttt_engine_set_cache(e, 0, 0);  // drop this engine's own table
    if (rc) return rc;
    e->cache = owner->cache;
    e->cache.ctr = e->d_cache_ctr;  // statistics stay per engine
    e->cache_log2 = owner->cache_log2;
    e->cache_clear_every = 0;       // only the owner clears
    e->cache_owner = false;
    return UTTT_OK;
}

int uttt_engine_cache_clear(uttt_engine_t *e) {
    if (!e) return UTTT_ERR_ARG;
    if (!e->cache.flag || !e->cache_owner) return UTTT_OK;
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipMemsetAsync(e->cache.flag, 0, sizeof(uint32_t) * ((size_t)1 << e->cache_log2), e->stream));
    // engines sharing the table launch on their own streams: nothing would order their next
    // lookups after this clear, so it completes before the call returns (once per run)
    HIP_TRY(hipStreamSynchronize(e->stream));
    return UTTT_OK;
}

int uttt_engine_cache_stats(uttt_engine_t *e, int64_t *hits, int64_t *misses, int64_t *inserts) {
    return uttt_engine_cache_stats2(e, hits, misses, inserts, nullptr);
}

int uttt_engine_cache_stats2(uttt_engine_t *e, int64_t *hits, int64_t *misses, int64_t *inserts,
                             int64_t *replacements) {
    if (!e) return UTTT_ERR_ARG;
    HIP_TRY(hipSetDevice(e->device));
    static thread_local unsigned long long raw[4 * kRow];
    HIP_TRY(hipMemcpyAsync(raw, e->d_cache_ctr, sizeof(raw), hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    unsigned long long c[4] = {0ull, 0ull, 0ull, 0ull};
    for (int k = 0; k < 4; ++k)
        for (int i = 0; i < kStripes; ++i) c[k] += raw[k * kRow + i * kStripeStride];
    if (hits) *hits = (int64_t)c[0];
    if (misses) *misses = (int64_t)c[1];
    if (inserts) *inserts = (int64_t)c[2];
    if (replacements) *replacements = (int64_t)c[3];
    return UTTT_OK;
}

// -------------------------------------------------------------- telemetry --
int uttt_engine_set_timing(uttt_engine_t *e, int32_t enabled) {
    if (!e) return UTTT_ERR_ARG;
    e->timing = enabled != 0;
    return UTTT_OK;
}

int uttt_engine_kernel_stats(uttt_engine_t *e, int32_t kernel, double *total_ms, int64_t *launches, int64_t *bytes) {
    if (!e || kernel < 0 || kernel >= kKernelCount) return UTTT_ERR_ARG;
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipStreamSynchronize(e->stream));
    drain_events(e);
    unsigned long long b[kRow];
    HIP_TRY(hipMemcpy(b, e->d_bytes + (size_t)kernel * kRow, sizeof(b), hipMemcpyDeviceToHost));
    unsigned long long sum = 0ull;
    for (int i = 0; i < kStripes; ++i) sum += b[i * kStripeStride];
    if (total_ms) *total_ms = e->ms[kernel];
    if (launches) *launches = e->launches[kernel];
    if (bytes) *bytes = (int64_t)sum;
    return UTTT_OK;
}

#ifdef UTTT_DIAG_BUILD
// Diagnostics engine build only: k_select's phase cycles (SelClock) summed over the first kSelDiagTrees
// trees, out[2 * kSpCount + 2]; reset zeroes them.
// the last k_select launch's per-tree wall-clock stamps (g_sel_rt): out[tree * 4 + {start, first root
// done, end, trips}], n_trees entries
int uttt_diag_select_pretouch(int32_t mode) {
    if (mode < 0 || mode > 3) return UTTT_ERR_ARG;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_sel_pretouch), &mode, sizeof(mode)) == hipSuccess ? UTTT_OK : UTTT_ERR_HIP;
}

int uttt_diag_select_rt(unsigned long long *out, int32_t n_trees) {
    static unsigned long long host[kSelDiagTrees][4];
    if (!out || n_trees < 0 || n_trees > kSelDiagTrees) return UTTT_ERR_ARG;
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_sel_rt), sizeof(host)) != hipSuccess) return UTTT_ERR_HIP;
    memcpy(out, host, sizeof(unsigned long long) * 4 * (size_t)n_trees);
    return UTTT_OK;
}

int uttt_diag_select_cycles(unsigned long long *out, int32_t reset) {
    static unsigned long long host[kSelDiagTrees][2 * kSpCount + 2];
    if (out) {
        if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_sel_cyc), sizeof(host)) != hipSuccess) return UTTT_ERR_HIP;
        for (int j = 0; j < 2 * kSpCount + 2; ++j) {
            out[j] = 0ull;
            for (int t = 0; t < kSelDiagTrees; ++t) out[j] += host[t][j];
        }
    }
    if (reset) {
        memset(host, 0, sizeof(host));
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_sel_cyc), host, sizeof(host)) != hipSuccess) return UTTT_ERR_HIP;
    }
    return UTTT_OK;
}
#endif

int uttt_engine_reset_stats(uttt_engine_t *e) {
    if (!e) return UTTT_ERR_ARG;
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipStreamSynchronize(e->stream));
    drain_events(e);
    for (int k = 0; k < kKernelCount; ++k) {
        e->ms[k] = 0.0;
        e->launches[k] = 0;
    }
    HIP_TRY(hipMemsetAsync(e->d_bytes, 0, sizeof(unsigned long long) * kKernelCount * kRow, e->stream));
    HIP_TRY(hipMemsetAsync(e->d_cache_ctr, 0, sizeof(unsigned long long) * 4 * kRow, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return UTTT_OK;
}

}  // extern "C"
