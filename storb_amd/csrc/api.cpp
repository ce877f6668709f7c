// api.cpp — the C ABI of libstorbec.so (declared in include/storb_ec.h).
//
// Replaces zfec's CPython extension on storb's path
// (/root/reference/storb/util/piece.py:8,129-130,196-197).  Responsibilities:
//   * validate exactly the preconditions zfec / easyfec enforce, returning
//     SEC_E* codes the Python layer maps to the same exceptions;
//   * build the per-batch launch plan (descriptors, tiles, tail items) on the
//     host and cache it, so a caller that repeats a batch shape (the
//     validator's steady state, bench.py) pays no host work or metadata upload;
//   * keep the coefficient tables device-resident, expanded on the GPU from
//     coefficient bytes (encode tables per (k, m), decode tables per erasure
//     pattern);
//   * SEC_F_HOST calls: stream the batch through pinned slabs on two pipeline
//     slots (gather -> H2D -> kernels -> D2H -> scatter), so host staging copies,
//     PCIe transfers in both directions and the kernels of different slabs overlap.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#include <algorithm>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "task_pool.hpp"
#include "bignum.hpp"
#include "gf_host.hpp"
#include "kernels.hpp"
#include "storb_ec.h"

namespace {

thread_local std::string g_hip_err;

int hip_fail(hipError_t e, const char *what)
{
    g_hip_err = std::string(what) + ": " + hipGetErrorString(e);
    return SEC_EHIP;
}

#define CK(x)                                   \
    do {                                        \
        hipError_t e_ = (x);                    \
        if (e_ != hipSuccess)                   \
            return hip_fail(e_, #x);            \
    } while (0)

#define RC(x)                 \
    do {                      \
        int rc_ = (x);        \
        if (rc_)              \
            return rc_;       \
    } while (0)

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes)
    {
        if (bytes <= cap)
            return SEC_OK;
        if (p)
            CK(hipFree(p));
        p = nullptr;
        cap = 0;
        size_t want = std::max(bytes, (size_t)1 << 16);
        if (hipMalloc(&p, want) != hipSuccess) {
            p = nullptr;
            return SEC_ENOMEM;
        }
        cap = want;
        return SEC_OK;
    }
    void release()
    {
        if (p)
            (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T> T *as(size_t off = 0) const { return reinterpret_cast<T *>((char *)p + off); }
};

// Process-wide pool of pinned host buffers (hipHostMalloc; page-locked and mapped for every
// device).  The staging buffers of host-mode calls (the pipeline slots' slabs, sec_encode_pieces'
// parity scratch) are borrowed from it for the call and given back when the call returns, so a
// context holds no locked memory between calls however many contexts a process opens (one per
// caller thread: engine.get_engine); the pool keeps at most kPinKeep bytes of idle buffers for
// the next call (reused without a new hipHostMalloc) and frees the rest, largest first.
// sec_host_pinned_bytes reports both figures.  The pool is never destroyed (its buffers go with
// the process), so no hipHostFree runs after the HIP runtime's teardown.
constexpr size_t kPinKeep = (size_t)512 << 20;
// Against contexts that keep their staging between calls (round 5), per call and on the 1 GiB
// streams: level within the boxes' spread (profiles/r06_pin_return_ab.txt).

class PinPool {
  public:
    static PinPool &get()
    {
        static PinPool *pool = new PinPool;
        return *pool;
    }
    // the smallest idle buffer of >= want bytes, else a new one; nullptr if hipHostMalloc fails
    void *take(size_t want, size_t *cap)
    {
        {
            std::lock_guard<std::mutex> lk(mu_);
            auto it = idle_.lower_bound(want);
            if (it != idle_.end()) {
                void *p = it->second;
                *cap = it->first;
                idle_bytes_ -= it->first;
                loaned_ += it->first;
                idle_.erase(it);
                return p;
            }
        }
        void *p = nullptr;
        if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess)
            return nullptr;
        std::lock_guard<std::mutex> lk(mu_);
        *cap = want;
        loaned_ += want;
        return p;
    }
    void give(void *p, size_t cap)
    {
        std::vector<void *> drop;
        {
            std::lock_guard<std::mutex> lk(mu_);
            loaned_ -= cap;
            idle_.emplace(cap, p);
            idle_bytes_ += cap;
            while (idle_bytes_ > kPinKeep && !idle_.empty()) {
                auto last = std::prev(idle_.end());
                idle_bytes_ -= last->first;
                drop.push_back(last->second);
                idle_.erase(last);
            }
        }
        for (void *q : drop)
            (void)hipHostFree(q);
    }
    void stats(int64_t *loaned, int64_t *idle)
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (loaned)
            *loaned = (int64_t)loaned_;
        if (idle)
            *idle = (int64_t)idle_bytes_;
    }

  private:
    std::mutex mu_;
    std::multimap<size_t, void *> idle_;
    size_t idle_bytes_ = 0, loaned_ = 0;
};

// A pinned host buffer.  pooled (default): borrowed from PinPool, given back by release();
// else its own hipHostMalloc (the context's small metadata staging).
struct PinBuf {
    void *p = nullptr;
    size_t cap = 0;
    bool pooled = true;
    int ensure(size_t bytes)
    {
        if (bytes <= cap)
            return SEC_OK;
        release();
        size_t want = std::max(bytes, (size_t)1 << 16);
        if (pooled) {
            p = PinPool::get().take(want, &cap);
            if (!p) {
                cap = 0;
                return SEC_ENOMEM;
            }
            return SEC_OK;
        }
        if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) {
            p = nullptr;
            return SEC_ENOMEM;
        }
        cap = want;
        return SEC_OK;
    }
    void release()
    {
        if (p) {
            if (pooled)
                PinPool::get().give(p, cap);
            else
                (void)hipHostFree(p);
        }
        p = nullptr;
        cap = 0;
    }
    char *c(size_t off = 0) const { return (char *)p + off; }
};

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// ---- context options (sec_ctx_set_option) --------------------------------------
// The plan rules below pick kernels, tile widths and host paths from measured defaults.  A
// test or an A/B tool that must force another choice sets it on ITS context through
// sec_ctx_set_option; the library reads no environment variable.  Setting an option drops the
// context's cached plans, so the next call is planned with it.  Names keep the SEC_ prefix the
// knobs had as environment variables in rounds 1-3 (tools/sweep.py variant strings use them).
// Round 5 pruned the options whose only use was an A/B against a plan that won (their kernels
// and results are in tools/archive/); what is left forces a SHIPPED path (tests) or sizes the
// host pipeline.
enum Opt {
    O_SYN,               // syndrome decodes: -1 cost rule, 0 off, 1 wherever they apply
    O_SYN_FUSED,         // 0: never the one-wave fused kernel
    O_SYN_RATIO,         // syndrome path taken under this many per mille of the direct estimate
    O_BS,                // bit-sliced encode: -1 rule (bs_shape), 0 off, 1 every shape it has
    O_BS_LANES,          // lanes of a bit-sliced / syndrome tile (64, 128, 256)
    O_SHA1_SPLIT,        // -1 rule, 0 one-lane kernel, 1 two-wave kernel
    O_SLAB_BYTES,        // host staging slab
    O_SLAB_BYTES_DIGEST, // host staging slab of SHA-1 / bignum calls
    O_COPY_THREADS,      // 0 rule, or host copy-pool threads
    O_REGISTER_MIN,      // page-lock pageable host buffers for calls moving >= this many bytes (0: never)
    O_HOST_JOIN,         // 0: the GPU writes every byte of a host reassembly
    O_COUNT
};

struct OptSpec {
    const char *name;
    int64_t dflt, lo, hi;
};

constexpr OptSpec kOpts[O_COUNT] = {
    {"SEC_SYN", -1, -1, 1},
    {"SEC_SYN_FUSED", 1, 0, 1},
    {"SEC_SYN_RATIO", 900, 1, 1000000},
    {"SEC_BS", -1, -1, 1},
    {"SEC_BS_LANES", 256, 64, 256},
    {"SEC_SHA1_SPLIT", -1, -1, 1},
    {"SEC_SLAB_BYTES", (int64_t)64 << 20, (int64_t)1 << 16, (int64_t)1 << 40},
    {"SEC_SLAB_BYTES_DIGEST", (int64_t)512 << 20, (int64_t)1 << 16, (int64_t)1 << 40},
    {"SEC_COPY_THREADS", 0, 0, 256},
    {"SEC_REGISTER_MIN", (int64_t)4 << 20, 0, (int64_t)1 << 62},
    {"SEC_HOST_JOIN", 1, 0, 1},
};

struct Options {
    int64_t v[O_COUNT];
    Options()
    {
        for (int i = 0; i < O_COUNT; ++i)
            v[i] = kOpts[i].dflt;
    }
    int64_t operator[](Opt o) const { return v[o]; }
    int lanes(Opt o) const { return (int)std::max<int64_t>(64, std::min<int64_t>(256, v[o])) / 64 * 64; }
};

int opt_index(const char *name)
{
    if (!name)
        return -1;
    for (int i = 0; i < O_COUNT; ++i)
        if (!strcmp(name, kOpts[i].name))
            return i;
    return -1;
}

// ---- plan ---------------------------------------------------------------
struct Group {
    int rows, U, lanes, wide;  // wide: k > kBatchVecs / U, blocks loaded in several batches
    uint32_t first, count;
    int mfma = 0;              // bin kind.  Encode: 3 = sec_encode_bs_kernel of shape `rows`, row group U;
                               // decode: the small-batch variant's batch (dec_small_kb), or 0
};

// One launch unit: all chunks (device mode) or one slab of chunks (host mode).
struct SubPlan {
    int64_t c0 = 0, c1 = 0;  // chunk range
    std::vector<Group> groups;
    size_t off_desc = 0, off_tiles = 0, off_tail = 0, off_soff = 0, off_srow = 0, off_mrow = 0, off_savail = 0;
    uint32_t ntail = 0;
    uint64_t in_bytes = 0, out_bytes = 0;  // dense slab sizes (host mode)
    size_t off_msgs = 0;                   // messages of this unit (SHA-1, bignum)
    uint32_t nmsgs = 0;
    bool sha_split = false;  // SHA-1 messages: the two-wave kernel (sha1_split)
    size_t off_segs = 0, off_seginfo = 0;  // bignum: segments of the messages, per-message (first, count)
    uint32_t nsegs = 0, max_seg = 0;       // segment count; most segments of one message
    uint64_t dig_first = 0;                // first digest slot of this unit
    uint64_t dig_off = 0;                  // host mode: digests' offset in the slab output
    // syndrome decodes (decode): phase 1 launches (bit-sliced syndromes) and phase 2 launches
    // (the Cauchy solve), one each per shape
    // (shape, (first, count)) in tiles; synf: the fused kernel (both phases in one wave)
    std::vector<std::pair<int, std::pair<uint32_t, uint32_t>>> syn1, syn2, synf;
    size_t off_sdesc = 0, off_stiles = 0, off_ssoff = 0, off_ssavail = 0, off_vdesc = 0, off_vtiles = 0,
           off_masks = 0, off_ftiles = 0;
    uint64_t syn_bytes = 0;  // syndrome scratch of this unit
    int syn_lanes = 256;     // lanes of the syndrome kernels' tiles (their span per tile)
};

struct Plan {
    std::vector<uint8_t> key;
    uint64_t gen = 0;  // table-cache generation the plan was built against
    std::vector<SubPlan> subs;
    DevBuf meta;  // device copy of the metadata image of every sub-plan
    bool valid = false;
    int64_t nsyn = 0, ndirect = 0, nfused = 0;  // decode: chunks with a lost primary, by method
};

// Device-resident GF coefficient tables (5 dwords per coefficient), keyed by
// matrix identity.  Reset (and generation bumped) when it outgrows its buffer.
struct TableCache {
    DevBuf buf;
    size_t used = 0;  // dwords
    uint64_t gen = 1;
    std::map<std::string, uint32_t> index;
};

struct PendingExpand {
    std::vector<uint8_t> coef;  // layout [input slot][output row]
    uint32_t dst;               // dword offset in the cache buffer
};

// Host-side image of the metadata, uploaded with one copy.
struct Image {
    std::vector<char> bytes;
    size_t put(const void *src, size_t n)
    {
        const size_t off = align_up(bytes.size(), 256);
        bytes.resize(off + n);
        if (n)
            memcpy(bytes.data() + off, src, n);
        return off;
    }
};

// Lanes of every U = 1 tile (U > 1 tiles are 256 lanes).  An encode batch whose blocks are all
// >= 64 KiB gets tiles one wave wide (1 KiB of each block per workgroup): in-process A/B
// (profiles/r02_enc_lanes.jsonl) C2 encode +1.9-2.0 %, RS(8,3) on 1 MiB chunks +2.3-2.6 %,
// zfec(16,24) even, while C4's 6554 B blocks lose 4.7 %; a mixed batch (C5) keeps one tile
// width, since its large chunks alone at 64 lanes (a second launch) cost it 9 %.  The 1:1
// copy behind a decode measured no gain from narrower tiles (-1 %).
int full_lanes(bool decode, bool narrow = false) { return !decode && narrow ? 64 : sec::kLanes; }

// One u-step (4 KiB of each block) per 256-lane tile: one 16 B vector per block and lane.
// Measured on C2 against U = 2 / 4: encode 6.48 vs 6.09 / 5.95 TB/s, decode 6.31 vs 5.79 / 5.62
// (profiles/r01_sweep_u.jsonl); round 5 stopped building the U > 1 kernels.
constexpr int kU = 1;

// Whether a group over k blocks runs in the wide (W) kernels, which load the blocks in several
// batches (kernels.hip SEC_WIDE_BATCH): k > kBatchVecs.  (Round 4's SEC_WIDE_K8 moved 8-row groups
// there from a lower k for A/B; its default, 16, is this same rule.)
bool is_wide(int k) { return k > sec::kBatchVecs; }

using Bins = std::map<std::tuple<int, int, int, int, int>, std::vector<sec::Tile>>;  // (kind, rows, U, lanes, wide)

uint64_t round64(uint64_t v) { return (v + 63) / 64 * 64; }

// Decodes that copy nothing (recover-only, and the copy-free host-join calls) of chunks with
// k <= 4 run a kernel variant whose load batch is 4 slots instead of 16: 57 instead of 104
// VGPRs, 8 waves per SIMD instead of 4.  Measured on C3 recover-only (tools/sweep.py
// --recover, env held during the timed calls): 6.42 against 5.91 TB/s; the same batches cost
// the reassembling decode 4 %, and 8-slot batches for k <= 8 measured 1.4 % slower on RS(8,3)
// recover-only (profiles/r02_dec_small_kb_ab.jsonl).
int dec_small_kb(int k) { return k <= 4 ? 4 : 0; }

// Syndrome decode (kernels_bs.hip) for a chunk that lost e data blocks, when its shape has the
// bit-sliced kernels: the one-wave kernel sec_decode_bs_kernel ("fused": e <= 16 and every
// present parity row in one 16-row group, the syndromes never leave the registers) or the two
// kernels sec_syndrome_bs_kernel + sec_solve_bs_kernel ("two": syndromes through HBM, any e).
// Chosen per chunk by a time estimate per 4 byte positions, each kernel taking the longer of its
// VALU issue time (ops / R, R the VALU rate it sustains) and its memory time (bytes / BW);
// both constants per kernel were fitted on the A/B (tools/syn_ab.py, profiles/r03_syn_ab.jsonl:
// fixed and random erasure patterns of zfec(64,96), (32,48), (16,24) and C4):
//   direct: ceil(e / 8) v_perm row groups (5 selector ops + 4.5 per row) over all k slots;
//           R 28 (1e12 lane-ops/s), BW 5.6 TB/s; reads k blocks, writes the chunk (or e rows);
//   fused:  phase 1 (k - e)(8.75 + e) + 15 e (bit-sliced rows of the present parity rows,
//           syndrome scaling), phase 2 2.75 e per touched 8-row group + e^2 + 14 e;
//           R 17, BW 5.0; the direct decode's bytes;
//   two:    phase 1 P (k - e) 8.75 + (k - e) e + 15 e over P touched parity groups, the data
//           read once per group (BW 5.0, or 4.0 when P = 2), or once when both groups share a
//           workgroup (sec_syndrome_bs_pair_kernel: BW 5.0); phase 2 2.75 e per touched 16-row group + e^2 + 14 e,
//           2 e rows of syndrome traffic; R 14.5.
// A syndrome path is taken when its estimate is under SEC_SYN_RATIO (default 900 per mille) of
// the direct one (970 for both-group chunks of one workgroup, below).  Options SEC_SYN = 0 / 1 turn the syndrome paths off / force them wherever they
// apply (fused where eligible); SEC_SYN_FUSED = 0 turns the fused kernel off.
double vperm_ops(int rows, int slots)
{
    double v = 0;
    for (int r = 0; r < rows; r += sec::kMaxRows)
        v += 5 + 4.5 * std::min(sec::kMaxRows, rows - r);
    return v * slots;
}

// Syndrome methods of a chunk (syn_choice).  (Round 4's one-kernel wave pair for both-group
// chunks, SEC_SYN_PAIR, tied the direct decode and is archived: tools/archive/.)
enum SynMethod { kSynTwo = 0, kSynFused = 1 };

// shape of the syndrome kernels for this chunk, or -1 (direct); `method`: two kernels or the
// one-wave fused kernel
int syn_choice(const Options &o, const sec_dec_chunk &c, const int *idx, int e, bool copies, int &method)
{
    method = kSynTwo;
    if (o[O_SYN] == 0)
        return -1;
    const int sh = sec_syn_shape(c.k, c.m);
    // e < k - 1: the LDS-ring kernels point an absent item's loads at the first present data block
    // other than the (possibly short) block k-1 (kernels_bs.hip item_addrs)
    if (sh < 0 || e < 1 || e >= c.k - 1 || c.B < 16 || c.B > 0xFFFFFFFFull - 8192 || c.padlen >= c.B)
        return -1;
    // g16: 16-row data groups with a lost row, the grouping the two-kernel estimate was fitted on
    // (r03); phase 2 now runs 8-row groups (SEC_SOLVE_NR), which measured faster, not slower, so
    // counting its groups would steer e > 16 chunks to the direct decode (r04_syn_ab_solve.jsonl)
    const int k = c.k, NR = sec_bs_rows(sh);
    uint64_t touched = 0, g8 = 0, g16 = 0;  // parity groups with a present row, data groups with a lost one
    for (int s = 0; s < k; ++s)
        if (idx[s] >= k) {
            touched |= 1ull << ((idx[s] - k) / NR);
            g8 |= 1ull << (s / 8);
            g16 |= 1ull << (s / 16);
        }
    const int P = __builtin_popcountll(touched);
    const bool can_fuse = P == 1 && e <= 16 && o[O_SYN_FUSED] != 0;
    if (o[O_SYN] == 1) {
        method = can_fuse ? kSynFused : kSynTwo;
        return sh;
    }
    auto t = [](double ops, double R, double bytes, double bw) { return std::max(ops / R, bytes / bw); };
    const double E = e, KE = k - e, out = copies ? k : e;
    const double direct = t(vperm_ops(e, k), 28, 4.0 * (k + out), 5.6);
    const double p2 = 2.75 * E * __builtin_popcountll(g16) + E * E + 14 * E;
    // both groups in one two-wave workgroup (sec_syndrome_bs_pair_kernel): the data read once
    // (1.07x at P = 2 instead of 1.45x), which fits the r04 A/B as P = 1's bytes and rate
    // (r04_syn_ab_final.jsonl)
    const bool wg2 = P == 2 && sec_syn_pair(sh);
    const double two = t(P * KE * 8.75 + KE * E + 15 * E, 14.5,
                         4.0 * (k + (wg2 ? 0 : (P - 1) * KE) + (copies ? KE : 0) + E), P > 1 && !wg2 ? 4.0 : 5.0) +
                       t(p2, 14.5, 4.0 * 2 * E, 5.0);
    const double fuse = can_fuse ? t(KE * (8.75 + E) + 15 * E + 2.75 * E * __builtin_popcountll(g8) + E * E + 14 * E,
                                     17, 4.0 * (k + out), 5.0)
                                 : 1e30;
    // margin: SEC_SYN_RATIO; at its default, 3 % for both-group chunks in one workgroup, whose
    // two and direct estimates fit the r04 A/B within 4 % (r04_syn_ab_final.jsonl: at e = 14 / 16
    // the two kernels beat the direct decode by 6-7 % at estimate ratios 0.96 / 0.92).  A caller
    // that sets SEC_SYN_RATIO gets exactly that margin for every chunk.
    const bool dflt_ratio = o[O_SYN_RATIO] == kOpts[O_SYN_RATIO].dflt;
    const int64_t ratio = wg2 && dflt_ratio ? 970 : o[O_SYN_RATIO];
    const double lim = (double)ratio / 1000.0 * direct;
    const double best = std::min(two, fuse);
    if (best >= lim)
        return -1;
    method = best == fuse ? kSynFused : kSynTwo;
    return sh;
}

// Work for one chunk.  `valid` = positions where every block is fully readable and
// every output row writable (the last data block's length, clamped to [0, B]).
// Tiles of 256 lanes x 4 KiB * U cover [0, valid); the ragged rest (and small chunks
// entirely) get U = 1 tiles of up to 1024 lanes sized to what is left, so a 64 KiB
// RS(10,4) chunk (6550 valid positions) is one 448-lane tile.  Lanes clamp to end at
// `valid`.  Positions [valid, B) (at most padlen for a normal chunk) are computed byte
// by byte by the last tile of each row group (Tile::ntail): a separate one-thread-per-
// byte launch cost C4 13-17 % on top of its main kernels (profiles/r01_c4_kernel_stats).
// Chunks with valid < 16 get no tile: all of [0, B) becomes one-thread tail items.
void add_work(Bins &bins, std::vector<sec::TailItem> &tail, uint32_t chunk, uint64_t B, int64_t valid, int rows_total,
              int k, bool decode, bool narrow = false, int small_kb = 0)
{
    if (B == 0)
        return;
    valid = std::max<int64_t>(0, std::min<int64_t>(valid, (int64_t)B));
    const uint64_t v = valid >= sec::kLaneBytes ? (uint64_t)valid : 0;
    const int ngroups = rows_total == 0 ? 1 : (rows_total + sec::kMaxRows - 1) / sec::kMaxRows;
    if (v == 0) {  // too small for a tile: every position is a tail item
        for (uint64_t t = 0; t < B; ++t)
            tail.push_back(sec::TailItem{chunk, (uint32_t)t});
        return;
    }
    const int wide = is_wide(k);
    for (int g = 0; g < ngroups; ++g) {
        const int r0 = g * sec::kMaxRows;
        const int rows = std::min(sec::kMaxRows, rows_total - r0);
        const int flanes = std::min(full_lanes(decode, narrow), sec::max_lanes(rows, kU));
        const uint64_t step = (uint64_t)sec::kLaneBytes * flanes * kU;
        // kind: 0, or the small-batch decode variant's batch (the group's kernel, see dec_small_kb)
        const int kind = small_kb && !wide && k <= small_kb ? small_kb : 0;
        auto &full = bins[{kind, rows, kU, flanes, wide}];
        // every tile is flanes wide, the chunk's last one with idle lanes past `valid`: one
        // launch per (rows, wide) class however mixed the chunk sizes are
        const uint64_t nfull = (v + step - 1) / step;
        for (uint64_t i = 0; i < nfull; ++i)
            full.push_back(sec::Tile{chunk, (uint32_t)(i * step), (uint32_t)r0, 0});
        full.back().ntail = (uint32_t)(B - v);  // the ragged end [v, B) rides on the last tile
    }
}

// Bit-sliced compile-time-matrix encode (kernels_bs.hip) for the shapes it is built for
// (C4's zfec(10,14), C5's (8,11), the policy's (8,12), (16,24), (32,48), (64,96)): every
// position [0, B) of a chunk with B >= 16, ragged end included, so such a chunk gets no
// sec_encode_kernel tile.  Tiles of SEC_BS_LANES lanes (default 256 = 8 KiB of each block).
// The shape of two row groups ((64,96): 2 x 16 rows) runs both groups of a span in one two-wave
// workgroup that shares each block's plane subsets through LDS (round 6; it replaced one launch
// interleaving runs of 8 tiles of each group so that the tiles reading the same blocks shared
// an XCD's L2: +3-16 %, profiles/r06_enc_ab.jsonl).  SEC_BS = 0 turns the kernel off (then the
// v_perm rows), SEC_BS = 1 uses it for every shape it has.  (The A/B forms -- one launch per
// group, (32,48) in 8-row groups, the interleaved launch, LDS-staged small chunks -- are
// archived: tools/archive/.)
constexpr int kBsPair = 98;       // Group::U of a two-wave launch, both row groups of a span per workgroup
#ifndef SEC_DEC_XCD_BIG
#define SEC_DEC_XCD_BIG 1  // the same order for the wide decodes' tiles (build knob, A/B; see build_decode_plan)
#endif
#ifndef SEC_PAIR_XCD_MIN_B
#define SEC_PAIR_XCD_MIN_B (3u << 20)  // the pair encode's XCD order from this block size (see flatten)
#endif
constexpr int kSolveLds = 1 << 16;  // phase-2 tile map keys of sec_solve_bs_lds_kernel launches
constexpr int kSynWg2 = 1 << 16;    // phase-1 tile map keys of sec_syndrome_bs_pair_kernel launches

int bs_shape(const Options &o, int k, int m, uint64_t B)
{
    if (o[O_BS] == 0)
        return -1;
    if (B < 16 || B > 0xFFFFFFFFull - 8192)
        return -1;
    // Default: the shapes with >= 8 parity rows, where the v_perm rows are VALU-bound (1.3-1.7x
    // here), and C4's RS(10,4) (+0-4 %, whole 65536-chunk job +2 %); the other p <= 4 shapes
    // measured 5-10 % slower here (C5's RS(8,3), zfec(8,12) on 4 MiB chunks; r02_bs_ab.jsonl)
    const int p = m - k;
    if (o[O_BS] != 1 && p < 8 && !(k == 10 && m == 14))
        return -1;
    return sec_bs_shape(k, m);
}

void add_bs_work(const Options &o, Bins &bins, uint32_t chunk, uint64_t B, int shape)
{
    if (sec_bs_groups(shape) > 1) {  // (64,96): one two-wave workgroup per span
        // (chunks of B >= SEC_PAIR_XCD_MIN_B in their own group, launched in XCD order: see flatten)
        auto &bin = bins[{3, shape, kBsPair, 128, B >= (uint64_t)SEC_PAIR_XCD_MIN_B ? 1 : 0}];
        for (uint64_t t0 = 0; t0 < B; t0 += sec_bs_span())
            bin.push_back(sec::Tile{chunk, (uint32_t)t0, 0, 0});
        return;
    }
    const int lanes = o.lanes(O_BS_LANES);
    const uint64_t step = (uint64_t)sec_bs_span() * (lanes / 64);
    auto &bin = bins[{3, shape, 0, lanes, 0}];
    for (uint64_t t0 = 0; t0 < B; t0 += step)
        bin.push_back(sec::Tile{chunk, (uint32_t)t0, 0, 0});
}

// XCD order.  Workgroup b of a launch is dispatched to XCD b % 8, so with the tiles in chunk
// order the eight XCDs interleave over the same region.  In XCD order each XCD instead walks
// one contiguous eighth of the group's tiles: tile(b) = start(b % 8) + b / 8 (bijective for
// any count).  Measured (profiles/r01_sweep2_*.jsonl): decode with full 256-lane multi-step
// tiles (C2/C3, U = 4) +2.6 %; encode within noise; one-tile-per-chunk groups (C4) -4 to
// -6 %; decode with the default U = 1 full tiles -3 % (profiles/r01_sweep_u1_knobs.jsonl).
// It paid only for decode groups of U > 1 tiles, which are no longer built, so it is off;
// SEC_XCD_ORDER = 1 (build knob, for A/B) applies it to every tile group of both kernels.
#ifndef SEC_XCD_ORDER
#define SEC_XCD_ORDER 0
#endif

// The zfec(64,96) pair encode of chunks with blocks of B >= 3 MiB runs its tiles in XCD order.
// In chunk order the ~512 resident workgroups cover about 1 MiB of each block row (2 KiB spans),
// so with 4 MiB blocks (storb's 256 MiB chunks) the 64 rows a span reads are 1 MiB windows at a
// 4 MiB stride and the concurrent addresses never vary the bits between: 3.82-4.01 TB/s, against
// 4.26 for B = 4032 KiB.  In XCD order each XCD walks its own eighth of the tiles, and 256 MiB
// chunks run 4.25-4.35 (+9-11 %); for 1 MiB-block (64 MiB) chunks, whose resident workgroups
// already cover whole rows, XCD order cost 4 %, so it stays off below 3 MiB
// (profiles/r06_enc_order_ab.jsonl).  SEC_PAIR_XCD_MIN_B (build knob, A/B; defined above add_bs_work).

bool use_xcd_order(bool, const Group &g) { return g.mfma < 3 && SEC_XCD_ORDER == 1; }

void xcd_order(std::vector<sec::Tile> &t)
{
    const size_t n = t.size(), q = n / 8, r = n % 8;
    if (n < 16)
        return;
    std::vector<sec::Tile> o(n);
    for (size_t b = 0; b < n; ++b) {
        const size_t x = b % 8;
        o[b] = t[x * q + std::min(x, r) + b / 8];
    }
    t.swap(o);
}

void flatten(const Bins &bins, std::vector<Group> &groups, std::vector<sec::Tile> &tiles, bool decode)
{
    groups.clear();
    for (auto &kv : bins) {
        if (kv.second.empty())
            continue;
        const size_t first = tiles.size();
        tiles.insert(tiles.end(), kv.second.begin(), kv.second.end());
        groups.push_back(Group{std::get<1>(kv.first), std::get<2>(kv.first), std::get<3>(kv.first),
                               std::get<4>(kv.first), (uint32_t)first, (uint32_t)(tiles.size() - first),
                               std::get<0>(kv.first)});
        if (use_xcd_order(decode, groups.back()) || (std::get<2>(kv.first) == kBsPair && std::get<4>(kv.first))) {
            std::vector<sec::Tile> g(tiles.begin() + first, tiles.end());
            xcd_order(g);
            std::copy(g.begin(), g.end(), tiles.begin() + first);
        }
    }
}

// Contiguous chunk ranges of at most `slab` input bytes (at least one chunk each).
std::vector<std::pair<int64_t, int64_t>> slabs_of(const std::vector<uint64_t> &in_bytes, size_t slab)
{
    std::vector<std::pair<int64_t, int64_t>> r;
    int64_t c0 = 0;
    uint64_t acc = 0;
    for (int64_t i = 0; i < (int64_t)in_bytes.size(); ++i) {
        if (i > c0 && acc + in_bytes[i] > slab) {
            r.emplace_back(c0, i);
            c0 = i;
            acc = 0;
        }
        acc += in_bytes[i];
    }
    if (c0 < (int64_t)in_bytes.size())
        r.emplace_back(c0, (int64_t)in_bytes.size());
    return r;
}

// ---- host pipeline slots ----------------------------------------------------
struct Slot {
    PinBuf in, out;
    DevBuf din, dout, dsyn;
    hipStream_t s = nullptr;
    hipEvent_t done = nullptr;
    bool busy = false;
    std::vector<sec::CopyJob> scatter;  // pinned out -> caller memory, once `done`
};

constexpr int kSlots = 2;

}  // namespace

struct sec_ctx {
    int device = 0;
    Options opt;  // sec_ctx_set_option
    hipStream_t own = nullptr;
    hipStream_t ext = nullptr;
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pending[4];
    std::vector<hipEvent_t> ev_pool;
    hipEvent_t stop_ev = nullptr;  // between timing_begin and timing_end of an attached launch
    PinBuf pin{nullptr, 0, false};  // metadata image staging (its own, not pooled: small, every call)
    hipEvent_t pin_ev = nullptr, meta_ev = nullptr;
    TableCache enc_tabs, dec_tabs;
    Plan enc_plan, dec_plan, sha_plan, bn_plan;
    DevBuf bn_scratch;  // host-mode staging of sec_bn_modexp / mulmod operands
    DevBuf bn_part;     // partial residues of segmented reductions (one region per slot)
    DevBuf syn;         // syndrome rows of device-mode syndrome decodes
    size_t bn_part_stride = 0;
    Slot slots[kSlots];
    // host threads (staging copies, joins, sec_encode_pieces' piece copies and SHA-1): the
    // process's pool of this context's size, shared with every other context of that size
    std::shared_ptr<sec::TaskPool> tasks;
    std::shared_ptr<sec::TaskPool> hash_tasks;  // sec_encode_pieces' piece copies + SHA-1 (SEC_HASH_POOL)
    // sec_encode_pieces: the parity of one sub-batch before its piece copies, two sub-batches in
    // turn, each at most max(SEC_SLAB_BYTES, one chunk's parity)
    PinBuf piece_par[2];
    // SEC_F_HOST encode / decode calls by path (sec_ctx_host_paths)
    int64_t zero_copy_calls = 0, registered_calls = 0, staged_calls = 0;
    int64_t syn_chunks = 0, direct_chunks = 0, fused_chunks = 0;  // decodes by method (sec_ctx_decode_paths)

    hipStream_t stream() const { return ext ? ext : own; }
    hipEvent_t ev()
    {
        if (!ev_pool.empty()) {
            hipEvent_t e = ev_pool.back();
            ev_pool.pop_back();
            return e;
        }
        hipEvent_t e = nullptr;
        (void)hipEventCreate(&e);
        return e;
    }
};

namespace {

int set_dev(const sec_ctx *ctx)
{
    CK(hipSetDevice(ctx->device));
    return SEC_OK;
}

// O_COPY_THREADS, or half the CPUs this process may use (affinity and cgroup quota), at most 7
int host_threads(const sec_ctx *ctx)
{
    return ctx->opt[O_COPY_THREADS] ? (int)ctx->opt[O_COPY_THREADS] : sec::default_pool_threads();
}

sec::TaskPool &tasks(sec_ctx *ctx)
{
    if (!ctx->tasks)
        ctx->tasks = sec::shared_pool(host_threads(ctx));
    return *ctx->tasks;
}

sec::TaskPool &pool(sec_ctx *ctx) { return tasks(ctx); }

// sec_encode_pieces' piece copies and SHA-1 ids run on a second shared pool of the usable CPUs but
// four (at most 12), the staging copies and joins staying on the 7-thread pool.  Against one
// pool for everything (16-CPU quota): the 1 GiB upload stream 5.0 -> 7.5-7.9 GiB/s, an 8 MiB
// chunk's encode + ids 1.2 -> 0.8 ms, C5 and the downloads level; one pool of 12-14 threads for
// everything throttled C5 instead (profiles/r06_hash_pool_ab.txt, r06_pool_threads_ab.txt).
// SEC_HASH_POOL (build knob, A/B): 0 = everything on the one pool.
#ifndef SEC_HASH_POOL
#define SEC_HASH_POOL 1
#endif
sec::TaskPool &hash_tasks(sec_ctx *ctx)
{
    if (!SEC_HASH_POOL || ctx->opt[O_COPY_THREADS])
        return tasks(ctx);
    if (!ctx->hash_tasks)
        ctx->hash_tasks = sec::shared_pool(std::min(12, std::max(1, sec::usable_cpus() - 4)));
    return *ctx->hash_tasks;
}

// The host-only joins (chunks with every primary present, a staged reassembly's present rows,
// sec_host_copy) run on the second pool too; the joins beside zero-copy kernels (C5's path) stay
// on the first.  The 1 GiB download stream with every data piece present 41-52 -> 53-69 GiB/s,
// C5's staged decode 14.5 -> 16-17.5, C5 itself and the upload level
// (profiles/r06_join_pool_ab.txt).  SEC_JOIN_POOL (build knob, A/B): 0 = on the first pool.
#ifndef SEC_JOIN_POOL
#define SEC_JOIN_POOL 1
#endif
sec::TaskPool &join_tasks(sec_ctx *ctx) { return SEC_JOIN_POOL ? hash_tasks(ctx) : tasks(ctx); }

int slots_init(sec_ctx *ctx)
{
    for (Slot &s : ctx->slots)
        if (!s.s) {
            CK(hipStreamCreateWithFlags(&s.s, hipStreamNonBlocking));
            CK(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
        }
    return SEC_OK;
}

// Finish a slot's in-flight slab: wait for its D2H, then scatter to caller memory.
int slot_retire(sec_ctx *ctx, Slot &s)
{
    if (!s.busy)
        return SEC_OK;
    s.busy = false;
    CK(hipEventSynchronize(s.done));
    pool(ctx).run_copies(s.scatter);
    s.scatter.clear();
    return SEC_OK;
}

int drain_all(sec_ctx *ctx)
{
    for (Slot &s : ctx->slots) {
        RC(slot_retire(ctx, s));
        if (s.s)
            CK(hipStreamSynchronize(s.s));
    }
    CK(hipStreamSynchronize(ctx->stream()));
    return SEC_OK;
}

// Make sure the pinned metadata staging is no longer read by an in-flight copy.
int pin_wait(sec_ctx *ctx)
{
    CK(hipEventSynchronize(ctx->pin_ev));
    return SEC_OK;
}

int table_ensure(TableCache &tc, const std::string &key, std::vector<uint8_t> &&coef,
                 std::vector<PendingExpand> &pending, uint32_t *off)
{
    auto it = tc.index.find(key);
    if (it != tc.index.end()) {
        *off = it->second;
        return SEC_OK;
    }
    const size_t need = coef.size() * sec::kTabDwords;
    if ((tc.used + need) * 4 > tc.buf.cap)
        return 1;  // caller resets the cache and retries
    *off = (uint32_t)tc.used;
    tc.index.emplace(key, *off);
    pending.push_back(PendingExpand{std::move(coef), *off});
    tc.used += need;
    return SEC_OK;
}

int table_reset(sec_ctx *ctx, TableCache &tc, size_t need_dwords)
{
    RC(drain_all(ctx));  // nothing may still read the old buffer
    size_t want = std::max<size_t>(tc.buf.cap * 2, std::max<size_t>(need_dwords * 4 * 2, (size_t)1 << 20));
    tc.buf.release();
    RC(tc.buf.ensure(want));
    tc.used = 0;
    tc.index.clear();
    ++tc.gen;
    return SEC_OK;
}

// Uploads the image with one H2D from pinned memory and expands new tables from
// the coefficient bytes placed at the end of the image.
int upload_plan(sec_ctx *ctx, Plan &plan, Image &img, TableCache &tc, const std::vector<PendingExpand> &pending)
{
    std::vector<size_t> coef_off;
    for (const auto &pe : pending)
        coef_off.push_back(img.put(pe.coef.data(), pe.coef.size()));
    const size_t bytes = img.bytes.size();
    RC(pin_wait(ctx));
    RC(ctx->pin.ensure(bytes));
    memcpy(ctx->pin.p, img.bytes.data(), bytes);
    RC(plan.meta.ensure(bytes));
    CK(hipMemcpyAsync(plan.meta.p, ctx->pin.p, bytes, hipMemcpyHostToDevice, ctx->stream()));
    CK(hipEventRecord(ctx->pin_ev, ctx->stream()));
    for (size_t i = 0; i < pending.size(); ++i) {
        int e = sec_launch_expand(plan.meta.as<uint8_t>(coef_off[i]), (uint32_t)pending[i].coef.size(),
                                  tc.buf.as<uint32_t>() + pending[i].dst, ctx->stream());
        if (e)
            return hip_fail((hipError_t)e, "sec_expand_tables");
    }
    return SEC_OK;
}

// Kernel timing (sec_ctx_set_timing).  Around the EC launchers (`attached`), the events ride
// on the kernels' own dispatch packets (sec_launch_events: the first launch records the
// start, the last the stop), so timing inserts no marker packets between back-to-back
// kernels: two hipEventRecord markers per launch measured 3-5 % off the bench's rate.  A
// call that launched nothing records both events at once (zero time); other launchers
// (bignum) get plain event records around them.
int timing_begin(sec_ctx *ctx, hipEvent_t *a, hipStream_t s, bool attached = true)
{
    *a = nullptr;
    if (!ctx->timing)
        return SEC_OK;
    *a = ctx->ev();
    if (attached) {
        ctx->stop_ev = ctx->ev();
        sec_launch_events(*a, ctx->stop_ev);
    } else {
        ctx->stop_ev = nullptr;
        CK(hipEventRecord(*a, s));
    }
    return SEC_OK;
}

int timing_end(sec_ctx *ctx, hipEvent_t a, int kind, hipStream_t s)
{
    if (!a)
        return SEC_OK;
    hipEvent_t b = ctx->stop_ev;
    ctx->stop_ev = nullptr;
    if (b) {
        if (sec_launch_events(nullptr, nullptr) == 0) {
            CK(hipEventRecord(a, s));
            CK(hipEventRecord(b, s));
        }
    } else {
        b = ctx->ev();
        CK(hipEventRecord(b, s));
    }
    ctx->pending[kind].emplace_back(a, b);
    return SEC_OK;
}

// SHA-1 kernel for a launch's messages: sec_sha1_split_kernel (message schedule on a second
// wave) when the messages are few and long, so the round chains are the bound; else one lane
// per message.  Option SEC_SHA1_SPLIT = 0 / 1 forces it.
bool sha1_split(const Options &o, const std::vector<sec::MsgDesc> &md)
{
    if (o[O_SHA1_SPLIT] >= 0)
        return o[O_SHA1_SPLIT] == 1;
    if (md.empty())
        return false;
    uint64_t blocks = 0;
    for (const sec::MsgDesc &m : md)
        blocks += m.len / 64;
    // measured (profiles/r02_sha1_split_ab.jsonl): faster up to 16384 messages of 64 KiB (256
    // one-lane waves), slower at 65536 x 16 KiB and C4's 114688 x 6554 B
    return md.size() <= ((size_t)16 << 10) && blocks / md.size() >= 256;  // >= 16 KiB on average
}

int check_sharenums(int k, int m, const int32_t *s)
{
    bool seen[256] = {false};
    for (int i = 0; i < k; ++i) {
        if (s[i] < 0 || s[i] >= m)
            return SEC_ESHARENUM;
        if (seen[s[i]])
            return SEC_EDUPSHARE;
        seen[s[i]] = true;
    }
    return SEC_OK;
}

uint64_t enc_B(const sec_enc_chunk &c) { return (c.n + (uint64_t)c.k - 1) / (uint64_t)c.k; }

// ---- encode plan ------------------------------------------------------------
// digest: 0 none, 1 every block's SHA-1 (sec_encode_digest_batch), 2 the parity blocks' only
// (sec_encode_pieces with SEC_F_GPU_PARITY_IDS: digest slot s of a chunk's m - k)
int build_encode_plan(sec_ctx *ctx, const sec_enc_chunk *chunks, int64_t nchunks, bool host, int digest)
{
    Plan &plan = ctx->enc_plan;
    TableCache &tc = ctx->enc_tabs;
    std::vector<PendingExpand> pending;
    std::vector<uint32_t> tab_of((size_t)nchunks, 0);
    for (int attempt = 0;; ++attempt) {
        pending.clear();
        size_t need = 0;
        bool overflow = false;
        std::map<std::pair<int, int>, uint32_t> local;
        for (int64_t i = 0; i < nchunks && !overflow; ++i) {
            const int k = chunks[i].k, m = chunks[i].m;
            if (m == k)
                continue;
            auto lk = local.find({k, m});
            if (lk != local.end()) {
                tab_of[i] = lk->second;
                continue;
            }
            const std::vector<uint8_t> enc = sec::encode_matrix(k, m);
            const int p = m - k;
            std::vector<uint8_t> coef((size_t)k * p);
            for (int j = 0; j < k; ++j)
                for (int r = 0; r < p; ++r)
                    coef[(size_t)j * p + r] = enc[(size_t)(k + r) * k + j];
            need += coef.size() * sec::kTabDwords;
            uint32_t off = 0;
            if (table_ensure(tc, std::to_string(k) + "/" + std::to_string(m), std::move(coef), pending, &off)) {
                overflow = true;
                break;
            }
            local[{k, m}] = off;
            tab_of[i] = off;
        }
        if (!overflow)
            break;
        if (attempt == 1)
            return SEC_ENOMEM;
        RC(table_reset(ctx, tc, need));
    }

    std::vector<std::pair<int64_t, int64_t>> ranges;
    if (host) {
        std::vector<uint64_t> ib((size_t)nchunks);
        for (int64_t i = 0; i < nchunks; ++i)
            ib[i] = chunks[i].n;
        // SHA-1 is one sequential chain per piece: a slab's hashing takes as long as
        // one piece, whatever the slab size, so digest mode uses few large slabs
        ranges = slabs_of(ib, (size_t)ctx->opt[digest ? O_SLAB_BYTES_DIGEST : O_SLAB_BYTES]);
    } else {
        ranges.emplace_back(0, nchunks);
    }
    Image img;
    plan.subs.clear();
    bool narrow = true;  // every block of the batch >= 64 KiB: one-wave encode tiles (full_lanes)
    for (int64_t i = 0; i < nchunks && narrow; ++i)
        if (chunks[i].m > chunks[i].k && enc_B(chunks[i]) < ((uint64_t)64 << 10))
            narrow = false;
    uint64_t dig = 0;
    for (auto [c0, c1] : ranges) {
        SubPlan sp;
        sp.c0 = c0;
        sp.c1 = c1;
        sp.dig_first = dig;
        std::vector<sec::EncDesc> descs((size_t)(c1 - c0));
        Bins bins;
        std::vector<sec::TailItem> tail;
        std::vector<sec::MsgDesc> msgs;
        for (int64_t i = c0; i < c1; ++i) {
            const sec_enc_chunk &c = chunks[i];
            const uint64_t B = enc_B(c);
            const int p = c.m - c.k;
            const int64_t valid = (int64_t)c.n - (int64_t)(c.k - 1) * (int64_t)B;
            sec::EncDesc &d = descs[i - c0];
            d.in_off = host ? sp.in_bytes : c.in_off;
            d.par_off = host ? sp.out_bytes : c.parity_off;
            d.par_stride = host ? B : c.parity_stride;
            d.B = (uint32_t)B;
            d.k = (uint32_t)c.k;
            d.p = (uint32_t)p;
            d.tab = tab_of[i];
            d.valid = (uint32_t)std::max<int64_t>(0, std::min<int64_t>(valid, (int64_t)B));
            d.pad = 0;
            if (digest) {  // data blocks from the input (padding synthesised), then parity
                for (int j = 0; j < c.k && digest == 1; ++j) {
                    const int64_t av = (int64_t)c.n - (int64_t)j * (int64_t)B;
                    msgs.push_back(sec::MsgDesc{d.in_off + (uint64_t)j * B, B,
                                                (uint64_t)std::max<int64_t>(0, std::min<int64_t>(av, (int64_t)B)), 0,
                                                0});
                }
                for (int r = 0; r < p; ++r)
                    msgs.push_back(sec::MsgDesc{d.par_off + (uint64_t)r * d.par_stride, B, B, 1, 0});
                dig += (uint64_t)(digest == 1 ? c.m : p);
            }
            sp.in_bytes += c.n;
            sp.out_bytes += (uint64_t)p * B;
            const int bs = p > 0 ? bs_shape(ctx->opt, c.k, c.m, B) : -1;
            if (bs >= 0)
                add_bs_work(ctx->opt, bins, (uint32_t)(i - c0), B, bs);
            else if (p > 0)
                add_work(bins, tail, (uint32_t)(i - c0), B, valid, p, c.k, false, narrow);
        }
        std::vector<sec::Tile> tiles;
        flatten(bins, sp.groups, tiles, false);
        sp.ntail = (uint32_t)tail.size();
        sp.nmsgs = (uint32_t)msgs.size();
        sp.sha_split = sha1_split(ctx->opt, msgs);
        sp.dig_off = sp.out_bytes;  // host mode: digests follow the slab's parity
        if (host)
            sp.out_bytes += (uint64_t)msgs.size() * 20;
        sp.off_desc = img.put(descs.data(), descs.size() * sizeof(sec::EncDesc));
        sp.off_tiles = img.put(tiles.data(), tiles.size() * sizeof(sec::Tile));
        sp.off_tail = img.put(tail.data(), tail.size() * sizeof(sec::TailItem));
        sp.off_msgs = img.put(msgs.data(), msgs.size() * sizeof(sec::MsgDesc));
        plan.subs.push_back(std::move(sp));
    }
    RC(upload_plan(ctx, plan, img, tc, pending));
    plan.gen = tc.gen;
    return SEC_OK;
}

int launch_encode_sub(sec_ctx *ctx, const Plan &plan, const SubPlan &sp, const uint8_t *in, uint8_t *par,
                      uint8_t *digests, hipStream_t s)
{
    const sec::EncDesc *dd = plan.meta.as<sec::EncDesc>(sp.off_desc);
    const sec::Tile *dt = plan.meta.as<sec::Tile>(sp.off_tiles);
    const uint32_t *tabs = ctx->enc_tabs.buf.as<uint32_t>();
    for (const Group &g : sp.groups) {
        int e = g.mfma == 3 ? sec_launch_encode_bs(g.rows, g.U == kBsPair ? -2 : g.U, g.lanes, in, par, dd,
                                                   dt + g.first, g.count, s)
                            : sec_launch_encode(g.rows, g.U, g.wide, g.lanes, in, par, dd, dt + g.first, g.count, tabs, s);
        if (e)
            return hip_fail((hipError_t)e, g.mfma == 3 ? "sec_encode_bs_kernel" : "sec_encode_kernel");
    }
    if (sp.ntail) {
        int e = sec_launch_encode_tail(in, par, dd, plan.meta.as<sec::TailItem>(sp.off_tail), sp.ntail, tabs, s);
        if (e)
            return hip_fail((hipError_t)e, "sec_encode_tail");
    }
    if (sp.nmsgs) {
        int e = sec_launch_sha1(in, par, plan.meta.as<sec::MsgDesc>(sp.off_msgs), sp.nmsgs, digests, s, sp.sha_split);
        if (e)
            return hip_fail((hipError_t)e, "sec_sha1_kernel");
    }
    return SEC_OK;
}

// ---- decode plan ------------------------------------------------------------
// Normalised slot order of every chunk (zfec's _fecmodule.c: primaries moved to
// their own slot); perm[i] = caller position of the block in normalised slot i.
struct DecLayout {
    std::vector<int> perm, idx;
    std::vector<uint64_t> first;  // per chunk: start in perm/idx
};

DecLayout dec_layout(const sec_dec_chunk *chunks, int64_t nchunks, const int32_t *sharenums)
{
    DecLayout L;
    L.first.resize((size_t)nchunks);
    std::vector<int> idx, perm;
    for (int64_t i = 0; i < nchunks; ++i) {
        const sec_dec_chunk &c = chunks[i];
        idx.assign(sharenums + c.slot0, sharenums + c.slot0 + c.k);
        sec::normalise_slots(c.k, idx, perm);
        L.first[i] = L.perm.size();
        L.perm.insert(L.perm.end(), perm.begin(), perm.end());
        L.idx.insert(L.idx.end(), idx.begin(), idx.end());
    }
    return L;
}

// Readable bytes of caller slot `j` of chunk c (sec_decode_batch_ex's block_avail; B if none).
uint64_t slot_avail(const sec_dec_chunk &c, const uint64_t *block_avail, int j)
{
    return block_avail ? std::min<uint64_t>(block_avail[c.slot0 + j], c.B) : c.B;
}

// Output bytes of a decode chunk: the reassembled chunk, or (recover-only) its e recovered
// blocks.  e = primaries absent from its sharenums.
uint64_t dec_nout(const sec_dec_chunk &c, const int32_t *sharenums, bool recover)
{
    if (!recover)
        return (uint64_t)c.k * c.B - c.padlen;
    uint64_t present = 0;
    for (int j = 0; j < c.k; ++j)
        present += sharenums[c.slot0 + j] < c.k;
    return ((uint64_t)c.k - present) * c.B;
}

// block_avail: nullable (device / zero-copy mode only: staged slots are zero-filled to B)
// nocopy (reassembly of host buffers, see sec_decode_batch_ex): recovered rows at their output
// rows as in a reassembly, but no present primary copied (the host copies those)
int build_decode_plan(sec_ctx *ctx, const sec_dec_chunk *chunks, int64_t nchunks, const uint64_t *block_offs,
                      const uint64_t *block_avail, const DecLayout &L, bool host, bool recover, bool nocopy = false)
{
    Plan &plan = ctx->dec_plan;
    TableCache &tc = ctx->dec_tabs;
    std::vector<PendingExpand> pending;
    std::vector<uint32_t> tab_of((size_t)nchunks, 0), e_of((size_t)nchunks, 0);
    std::vector<int> syn_of((size_t)nchunks, -1);  // syndrome-decode shape, or -1 (syn_choice)
    std::vector<char> fuse_of((size_t)nchunks, 0);  // ... its SynMethod
    for (int attempt = 0;; ++attempt) {
        pending.clear();
        size_t need = 0;
        bool overflow = false;
        for (int64_t i = 0; i < nchunks && !overflow; ++i) {
            const sec_dec_chunk &c = chunks[i];
            const int k = c.k;
            const int *idx = &L.idx[L.first[i]];
            std::vector<int> miss;
            for (int s = 0; s < k; ++s)
                if (idx[s] >= k)
                    miss.push_back(s);
            e_of[i] = (uint32_t)miss.size();
            if (miss.empty())
                continue;
            // the syndrome kernel reads every slot but data block k-1 whole (that one may be short:
            // zfec's padded block read in place)
            bool whole = true;
            for (int s = 0; s < k && whole && !host; ++s)
                whole = idx[s] == k - 1 || slot_avail(c, block_avail, L.perm[L.first[i] + s]) >= c.B;
            int fz = kSynTwo;
            const int sh = syn_of[i] =
                whole ? syn_choice(ctx->opt, c, idx, (int)miss.size(), !recover && !nocopy, fz) : -1;
            fuse_of[i] = fz;
            if (sh >= 0)
                continue;  // the syndrome path's matrices are compile-time (its scalings: the plan image)
            std::string key = std::to_string(k) + "/" + std::to_string(c.m) + ":";
            for (int s = 0; s < k; ++s)
                key += std::to_string(idx[s]) + ",";
            auto it = tc.index.find(key);
            if (it != tc.index.end()) {
                tab_of[i] = it->second;
                continue;
            }
            const int e = (int)miss.size();
            std::vector<uint8_t> coef;
            {
                std::vector<int> iv(idx, idx + k);
                std::vector<uint8_t> minv;
                if (!sec::decode_matrix(k, c.m, iv, minv))
                    return SEC_ESINGULAR;
                coef.resize((size_t)k * e);
                for (int s = 0; s < k; ++s)
                    for (int r = 0; r < e; ++r)
                        coef[(size_t)s * e + r] = minv[(size_t)miss[r] * k + s];
            }
            need += coef.size() * sec::kTabDwords;
            uint32_t off = 0;
            if (table_ensure(tc, key, std::move(coef), pending, &off)) {
                overflow = true;
                break;
            }
            tab_of[i] = off;
        }
        if (!overflow)
            break;
        if (attempt == 1)
            return SEC_ENOMEM;
        RC(table_reset(ctx, tc, need * 2 + ((size_t)1 << 18)));
    }

    plan.nsyn = plan.ndirect = plan.nfused = 0;
    for (int64_t i = 0; i < nchunks; ++i)
        if (e_of[i]) {
            ++(syn_of[i] >= 0 ? plan.nsyn : plan.ndirect);
            plan.nfused += syn_of[i] >= 0 && fuse_of[i] == kSynFused;
        }
    std::vector<std::pair<int64_t, int64_t>> ranges;
    if (host) {
        std::vector<uint64_t> ib((size_t)nchunks);
        for (int64_t i = 0; i < nchunks; ++i)
            ib[i] = (uint64_t)chunks[i].k * chunks[i].B;
        ranges = slabs_of(ib, (size_t)ctx->opt[O_SLAB_BYTES]);
    } else {
        ranges.emplace_back(0, nchunks);
    }
    Image img;
    plan.subs.clear();
    for (auto [c0, c1] : ranges) {
        SubPlan sp;
        sp.c0 = c0;
        sp.c1 = c1;
        // the syndrome tiles' span is built for this lane count; the launches take it from here
        const int syn_lanes = sp.syn_lanes = ctx->opt.lanes(O_BS_LANES);
        std::vector<sec::DecDesc> descs((size_t)(c1 - c0));
        std::vector<uint64_t> soff;
        std::vector<uint32_t> srow, mrow, savail;
        Bins bins;
        std::vector<sec::TailItem> tail;
        // syndrome decodes: phase-1 descriptors, slots and tiles, phase-2 descriptors and tiles
        // (tiles per shape), the scalings of both
        std::vector<sec::SynDesc> sdescs;
        std::vector<uint64_t> ssoff;
        std::vector<uint32_t> ssavail;
        std::map<int, std::vector<sec::Tile>> stiles, vtiles, ftiles;
        std::vector<sec::SolveDesc> vdescs;
        std::vector<uint64_t> masks;                                    // w / z scalings (scale_mask)
        std::map<std::string, std::pair<uint32_t, uint32_t>> mask_of;  // pattern -> (wq0, zq0)
        for (int64_t i = c0; i < c1; ++i) {
            const sec_dec_chunk &c = chunks[i];
            const uint64_t base = L.first[i];
            const int *idx = &L.idx[base];
            const uint32_t slot0 = (uint32_t)soff.size();
            std::vector<uint32_t> mr;
            uint64_t min_avail = c.B;
            for (int s = 0; s < c.k; ++s) {
                const int from = L.perm[base + s];
                soff.push_back(host ? sp.in_bytes + (uint64_t)s * c.B : block_offs[c.slot0 + from]);
                // recover-only: no copies, and recovered row r goes to output row r
                srow.push_back(!recover && !nocopy && idx[s] < c.k ? (uint32_t)idx[s] : 0xFFFFFFFFu);
                const uint64_t av = host ? c.B : slot_avail(c, block_avail, from);
                savail.push_back((uint32_t)av);
                min_avail = std::min(min_avail, av);
                if (idx[s] >= c.k)
                    mr.push_back(recover ? (uint32_t)mr.size() : (uint32_t)s);
            }
            mr.resize((size_t)c.k, 0);
            mrow.insert(mrow.end(), mr.begin(), mr.end());
            const uint64_t nout = recover ? (uint64_t)e_of[i] * c.B : (uint64_t)c.k * c.B - c.padlen;
            // positions below `valid`: every output row writable (the last one is the shortest)
            // and every slot readable; [valid, B) goes byte by byte, reading past avail as zero
            const int64_t valid = std::min<int64_t>(
                recover ? (int64_t)c.B : (int64_t)nout - (int64_t)(c.k - 1) * (int64_t)c.B, (int64_t)min_avail);
            sec::DecDesc &d = descs[i - c0];
            d.out_off = host ? sp.out_bytes : c.out_off;
            d.n = nout;
            d.B = (uint32_t)c.B;
            d.k = (uint32_t)c.k;
            d.e = e_of[i];
            d.tab = tab_of[i];
            d.slot0 = slot0;
            d.valid = (uint32_t)std::max<int64_t>(0, std::min<int64_t>(valid, (int64_t)c.B));
            sp.in_bytes += (uint64_t)c.k * c.B;
            sp.out_bytes += nout;
            const int sh = syn_of[i];
            if (sh >= 0 && nout > 0) {
                // phase 1: every present block in place, syndromes to the scratch
                const int k = c.k, p = c.m - c.k, e = (int)e_of[i], NR = sec_bs_rows(sh);
                const bool copies = !recover && !nocopy;
                sec::SynDesc sd{};
                sd.out_off = d.out_off;
                sd.syn_off = sp.syn_bytes;
                sd.B = (uint32_t)c.B;
                sd.last = recover ? (uint32_t)c.B : (uint32_t)(nout - (uint64_t)(k - 1) * c.B);
                sd.slot0 = (uint32_t)ssoff.size();
                ssoff.resize(ssoff.size() + (size_t)(k + p), 0);
                ssavail.resize(ssavail.size() + (size_t)(k + p), 0);
                for (int s = 0; s < k; ++s) {
                    const size_t j = sd.slot0 + (idx[s] < k ? (size_t)s : (size_t)idx[s]);
                    (idx[s] < k ? sd.dmask : sd.pmask) |= 1ull << (idx[s] < k ? s : idx[s] - k);
                    ssoff[j] = soff[slot0 + s];
                    ssavail[j] = savail[slot0 + s];
                }
                std::vector<int> gs;  // touched row groups, ascending
                for (int g = 0; g * NR < p; ++g)
                    if ((sd.pmask >> (g * NR)) & ((NR >= 64 ? ~0ull : (1ull << NR) - 1)))
                        gs.push_back(g);
                const int method = fuse_of[i];  // syn_choice: both phases in one kernel unless kSynTwo
                if (method == kSynTwo)
                    sp.syn_bytes += (uint64_t)e * sec::syn_stride(c.B);
                // the scalings of this erasure pattern (shared by the chunks that have it)
                uint64_t lost = 0;
                std::string key = std::to_string(k) + "/" + std::to_string(c.m) + ":";
                for (int s = 0; s < k; ++s) {
                    key += std::to_string(idx[s]) + ",";
                    if (idx[s] >= k)
                        lost |= 1ull << s;
                }
                auto mk = mask_of.find(key);
                if (mk == mask_of.end()) {
                    std::vector<int> S, Lost;
                    for (int r = 0; r < p; ++r)
                        if ((sd.pmask >> r) & 1)
                            S.push_back(r);
                    for (int s = 0; s < k; ++s)
                        if ((lost >> s) & 1)
                            Lost.push_back(s);
                    std::vector<uint8_t> w, z;
                    sec::cauchy_scales(k, S, Lost, w, z);
                    const std::pair<uint32_t, uint32_t> at{(uint32_t)masks.size(), (uint32_t)(masks.size() + e)};
                    for (uint8_t v : w)
                        masks.push_back(sec::scale_mask(v));
                    for (uint8_t v : z)
                        masks.push_back(sec::scale_mask(v));
                    mk = mask_of.emplace(key, at).first;
                }
                sd.wq0 = mk->second.first;
                sd.zq0 = mk->second.second;
                sd.flags = recover ? 2u : 0u;
                const uint32_t si = (uint32_t)sdescs.size();
                sdescs.push_back(sd);
                const uint64_t step = (uint64_t)sec_bs_span() * (syn_lanes / 64);
                if (method == kSynFused) {
                    auto &ft = ftiles[sh];
                    for (uint64_t t = 0; t < c.B; t += step)
                        ft.push_back(sec::Tile{si, (uint32_t)t, (uint32_t)(gs[0] * NR), copies ? 1u : 0u});
                    continue;
                }
                if (gs.size() == 2 && sec_syn_pair(sh)) {  // both groups, one two-wave workgroup per span
                    auto &st2 = stiles[kSynWg2 + sh];
                    for (uint64_t t = 0; t < c.B; t += sec_bs_span())
                        st2.push_back(sec::Tile{si, (uint32_t)t, 0u, copies ? 1u : 0u});
                } else {
                    auto &st = stiles[sh];
                    for (uint64_t t0 = 0; t0 < c.B; t0 += 8 * step)  // runs of 8 positions per group: one XCD
                        for (int g : gs)
                            for (uint64_t t = t0; t < std::min<uint64_t>(c.B, t0 + 8 * step); t += step)
                                st.push_back(
                                    sec::Tile{si, (uint32_t)t, (uint32_t)(g * NR), copies && g == gs[0] ? 1u : 0u});
                }
                // phase 2: the groups of lost rows, their tiles interleaved as phase 1's
                sec::SolveDesc vd{};
                vd.out_off = d.out_off;
                vd.syn_off = sd.syn_off;
                vd.lost = lost;
                vd.pmask = sd.pmask;
                vd.B = (uint32_t)c.B;
                vd.last = recover ? (uint32_t)c.B : (uint32_t)(nout - (uint64_t)(k - 1) * c.B);
                vd.zq0 = mk->second.second;
                vd.recover = recover ? 1u : 0u;
                const uint32_t vi = (uint32_t)vdescs.size();
                vdescs.push_back(vd);
                if (sec_solve_lds(sh)) {  // one workgroup per span, syndromes in LDS
                    auto &vt = vtiles[kSolveLds + sh * 64 + ((e + 7) / 8) * 8];
                    for (uint64_t t = 0; t < c.B; t += sec_bs_span())
                        vt.push_back(sec::Tile{vi, (uint32_t)t, 0u, 0u});
                    continue;
                }
                const int NR2 = sec_solve_rows(sh);
                std::vector<int> gl;
                for (int g = 0; g * NR2 < k; ++g)
                    if ((lost >> (g * NR2)) & ((NR2 >= 64 ? ~0ull : (1ull << NR2) - 1)))
                        gl.push_back(g);
                auto &vt = vtiles[sh];
                for (uint64_t t0 = 0; t0 < c.B; t0 += 8 * step)
                    for (int g : gl)
                        for (uint64_t t = t0; t < std::min<uint64_t>(c.B, t0 + 8 * step); t += step)
                            vt.push_back(sec::Tile{vi, (uint32_t)t, (uint32_t)(g * NR2), 0u});
            } else if (nout > 0 && !(nocopy && e_of[i] == 0)) {
                add_work(bins, tail, (uint32_t)(i - c0), c.B, valid, (int)e_of[i], c.k, true, false,
                         recover || nocopy ? dec_small_kb(c.k) : 0);
            }
        }
        // The two-kernel wide decode's tiles (phase 1 pairs, phase 2 LDS spans) in XCD order when
        // their blocks are large, as the pair encode's (add_bs_work): zfec(64,96) on 256 MiB chunks,
        // 32 lost 2.24 -> 2.39 TB/s, 24 random 2.51 -> 2.69; the one-wave fused path lost 8 % to it
        // and keeps chunk order (profiles/r06_dec_order_ab.jsonl).
        if (SEC_DEC_XCD_BIG) {
            auto big = [&](const std::vector<sec::Tile> &t, auto B_of) {
                for (const sec::Tile &x : t)
                    if (B_of(x) >= (uint64_t)SEC_PAIR_XCD_MIN_B)
                        return true;
                return false;
            };
            auto sB = [&](const sec::Tile &x) { return (uint64_t)sdescs[x.chunk].B; };
            auto vB = [&](const sec::Tile &x) { return (uint64_t)vdescs[x.chunk].B; };
            for (auto &kv : stiles)
                if (kv.first >= kSynWg2 && big(kv.second, sB))
                    xcd_order(kv.second);
            for (auto &kv : vtiles)
                if (kv.first >= kSolveLds && big(kv.second, vB))
                    xcd_order(kv.second);
        }
        std::vector<sec::Tile> tiles, stl, vtl;
        flatten(bins, sp.groups, tiles, true);
        for (auto &kv : stiles) {
            sp.syn1.push_back({kv.first, {(uint32_t)stl.size(), (uint32_t)kv.second.size()}});
            stl.insert(stl.end(), kv.second.begin(), kv.second.end());
        }
        for (auto &kv : vtiles) {
            sp.syn2.push_back({kv.first, {(uint32_t)vtl.size(), (uint32_t)kv.second.size()}});
            vtl.insert(vtl.end(), kv.second.begin(), kv.second.end());
        }
        std::vector<sec::Tile> ftl;
        for (auto &kv : ftiles) {
            sp.synf.push_back({kv.first, {(uint32_t)ftl.size(), (uint32_t)kv.second.size()}});
            ftl.insert(ftl.end(), kv.second.begin(), kv.second.end());
        }
        sp.off_ftiles = img.put(ftl.data(), ftl.size() * sizeof(sec::Tile));
        sp.off_sdesc = img.put(sdescs.data(), sdescs.size() * sizeof(sec::SynDesc));
        sp.off_stiles = img.put(stl.data(), stl.size() * sizeof(sec::Tile));
        sp.off_ssoff = img.put(ssoff.data(), ssoff.size() * 8);
        sp.off_ssavail = img.put(ssavail.data(), ssavail.size() * 4);
        sp.off_vdesc = img.put(vdescs.data(), vdescs.size() * sizeof(sec::SolveDesc));
        sp.off_vtiles = img.put(vtl.data(), vtl.size() * sizeof(sec::Tile));
        sp.off_masks = img.put(masks.data(), masks.size() * 8);
        sp.ntail = (uint32_t)tail.size();
        sp.off_desc = img.put(descs.data(), descs.size() * sizeof(sec::DecDesc));
        sp.off_tiles = img.put(tiles.data(), tiles.size() * sizeof(sec::Tile));
        sp.off_tail = img.put(tail.data(), tail.size() * sizeof(sec::TailItem));
        soff.resize(soff.size() + sec::kBatchVecs, 0);  // the kernels load a batch's offsets unconditionally
        sp.off_soff = img.put(soff.data(), soff.size() * 8);
        sp.off_srow = img.put(srow.data(), srow.size() * 4);
        sp.off_mrow = img.put(mrow.data(), mrow.size() * 4);
        sp.off_savail = img.put(savail.data(), savail.size() * 4);
        plan.subs.push_back(std::move(sp));
    }
    RC(upload_plan(ctx, plan, img, tc, pending));
    plan.gen = tc.gen;
    return SEC_OK;
}

int launch_decode_sub(sec_ctx *ctx, const Plan &plan, const SubPlan &sp, const uint8_t *blocks, uint8_t *out,
                      hipStream_t s, uint8_t *syn = nullptr)
{
    const sec::DecDesc *dd = plan.meta.as<sec::DecDesc>(sp.off_desc);
    const sec::Tile *dt = plan.meta.as<sec::Tile>(sp.off_tiles);
    const uint32_t *tabs = ctx->dec_tabs.buf.as<uint32_t>();
    const sec::DecSlots sl{plan.meta.as<uint64_t>(sp.off_soff), plan.meta.as<uint32_t>(sp.off_srow),
                           plan.meta.as<uint32_t>(sp.off_mrow), plan.meta.as<uint32_t>(sp.off_savail)};
    for (const Group &g : sp.groups) {
        // decode groups: the bin kind is the small-batch variant's batch (or 0)
        int e = sec_launch_decode(g.rows, g.U, g.wide, g.lanes, blocks, out, dd, dt + g.first, g.count, tabs, sl, s,
                                  g.mfma);
        if (e)
            return hip_fail((hipError_t)e, "sec_decode_kernel");
    }
    if (sp.ntail) {
        int e = sec_launch_decode_tail(blocks, out, dd, plan.meta.as<sec::TailItem>(sp.off_tail), sp.ntail, tabs,
                                       sl, s);
        if (e)
            return hip_fail((hipError_t)e, "sec_decode_tail");
    }
    if (sp.syn1.empty() && sp.synf.empty())
        return SEC_OK;
    if (!syn && !sp.syn1.empty())
        return SEC_EINVAL;
    // syndrome decodes: phase 1 (scaled syndromes + present primaries' copies), then phase 2
    // (the Cauchy solve) on the syndrome planes, in stream order
    const uint64_t *masks = plan.meta.as<uint64_t>(sp.off_masks);
    const sec::SynDesc *sd = plan.meta.as<sec::SynDesc>(sp.off_sdesc);
    const sec::Tile *st = plan.meta.as<sec::Tile>(sp.off_stiles);
    const sec::SynSlots ss{plan.meta.as<uint64_t>(sp.off_ssoff), plan.meta.as<uint32_t>(sp.off_ssavail), masks};
    const int lanes = sp.syn_lanes;  // what the plan's tiles were built for
    const sec::Tile *ft = plan.meta.as<sec::Tile>(sp.off_ftiles);
    for (const auto &g : sp.synf) {
        int e = sec_launch_decode_bs(g.first, lanes, blocks, out, sd, ft + g.second.first, g.second.second, ss, s);
        if (e)
            return hip_fail((hipError_t)e, "sec_decode_bs_kernel");
    }
    for (const auto &g : sp.syn1) {
        const bool wg2 = g.first >= kSynWg2;  // key kSynWg2 + shape: two-wave workgroups, both groups
        int e = wg2 ? sec_launch_syndrome_bs_pair(g.first - kSynWg2, blocks, out, syn, sd, st + g.second.first,
                                                  g.second.second, ss, s)
                    : sec_launch_syndrome_bs(g.first, lanes, blocks, out, syn, sd, st + g.second.first,
                                             g.second.second, ss, s);
        if (e)
            return hip_fail((hipError_t)e, wg2 ? "sec_syndrome_bs_pair_kernel" : "sec_syndrome_bs_kernel");
    }
    const sec::SolveDesc *vd = plan.meta.as<sec::SolveDesc>(sp.off_vdesc);
    const sec::Tile *vt = plan.meta.as<sec::Tile>(sp.off_vtiles);
    for (const auto &g : sp.syn2) {
        const bool staged = g.first >= kSolveLds;  // key kSolveLds + shape * 64 + LDS rows
        int e = staged ? sec_launch_solve_bs_lds((g.first - kSolveLds) / 64, (g.first - kSolveLds) % 64, syn, out, vd,
                                                 vt + g.second.first, g.second.second, masks, s)
                       : sec_launch_solve_bs(g.first, lanes, syn, out, vd, vt + g.second.first, g.second.second, masks, s);
        if (e)
            return hip_fail((hipError_t)e, staged ? "sec_solve_bs_lds_kernel" : "sec_solve_bs_kernel");
    }
    return SEC_OK;
}

// ---- pinned caller memory: the zero-copy host path ----------------------------
// A SEC_F_HOST encode / decode whose caller buffers all lie in page-locked host memory the
// HIP runtime maps at the same address on the device (hipHostMalloc / sec_host_alloc,
// hipHostRegister / sec_host_register) skips the staging pipeline: the device-mode kernels
// run straight on the host buffers and read / write them over PCIe, with no staging copy
// and no DMA.  Measured on C2 (tools/e2e_study.py): encode 50.9 GiB/s and decode 41.2 GiB/s
// against 33.4 / 17.5 staged, with the link's own H2D 53.6 and both-ways 45.2 GiB/s.
// Pageable memory keeps the staged path.
struct PinnedRange {
    uintptr_t lo = 0, hi = 0;  // last allocation found: [lo, hi)
};

// True when [p, p + len) lies inside ONE pinned allocation whose device address equals its
// host address.  `cache` remembers the last allocation so runs of blocks inside one buffer
// cost one lookup.  A failed lookup's error is cleared so later launches do not report it.
// (addresses arrive as base + offset integers: a NULL base with absolute offsets is legal in
// this ABI, and pointer arithmetic on NULL would let the compiler fold the NULL test away)
bool pinned(uintptr_t a, uint64_t len, PinnedRange *cache)
{
    const void *p = (const void *)a;
    if (len == 0)
        return true;
    if (!a)
        return false;
    if (cache->hi && a >= cache->lo && a + len <= cache->hi)
        return true;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    if (at.type != hipMemoryTypeHost || at.devicePointer != at.hostPointer || !at.devicePointer)
        return false;
    void *start = nullptr;
    size_t size = 0;
    if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, (hipDeviceptr_t)p) != hipSuccess ||
        hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, (hipDeviceptr_t)p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    const uintptr_t lo = (uintptr_t)start, hi = lo + size;
    if (!size || a < lo || a + len > hi)
        return false;
    cache->lo = lo;
    cache->hi = hi;
    return true;
}

// ---- host pipeline ----------------------------------------------------------
// For each slab: (CPU) gather caller bytes into the slot's pinned `in`; (slot stream) the
// kernels, then the scatter of pinned `out` into caller memory when the slot is next needed
// or at the end.  Two slots, so the CPU gathers slab i+1 and scatters slab i-1 while the GPU
// works on slab i.
// `direct`: the EC kernels run on the pinned slabs themselves (mapped at the same address on
// the device), reading and writing them over PCIe as the zero-copy path does, with no DMA
// copies.  A small call then costs its two host copies and one kernel, not two DMA
// round trips as well.  SHA-1 and the bignum kernels (one latency-bound lane or wave per
// message) keep the DMA into device scratch: every PCIe read would stall their chains.
bool pinned_mapped(const PinBuf &b)
{
    PinnedRange cache;
    return b.p && pinned((uintptr_t)b.p, b.cap, &cache);
}

template <class Gather, class Scatter, class Launch>
int run_pipeline(sec_ctx *ctx, Plan &plan, Gather gather, Scatter scatter, Launch launch, bool direct = false)
{
    RC(slots_init(ctx));
    CK(hipEventRecord(ctx->meta_ev, ctx->stream()));  // behind the plan upload / table expansion
    size_t i = 0;
    for (const SubPlan &sp : plan.subs) {
        Slot &sl = ctx->slots[i++ % kSlots];
        RC(slot_retire(ctx, sl));
        RC(sl.in.ensure(sp.in_bytes));
        RC(sl.out.ensure(sp.out_bytes));
        const bool on_pins = direct && pinned_mapped(sl.in) && pinned_mapped(sl.out);
        if (!on_pins) {
            RC(sl.din.ensure(sp.in_bytes));
            RC(sl.dout.ensure(sp.out_bytes));
        }
        std::vector<sec::CopyJob> jobs;
        gather(sp, sl.in.c(), jobs);
        pool(ctx).run_copies(jobs);
        CK(hipStreamWaitEvent(sl.s, ctx->meta_ev, 0));
        if (on_pins) {
            RC(launch(sp, (uint8_t *)sl.in.p, (uint8_t *)sl.out.p, sl.s));
        } else {
            CK(hipMemcpyAsync(sl.din.p, sl.in.p, sp.in_bytes, hipMemcpyHostToDevice, sl.s));
            RC(launch(sp, sl.din.as<uint8_t>(), sl.dout.as<uint8_t>(), sl.s));
            CK(hipMemcpyAsync(sl.out.p, sl.dout.p, sp.out_bytes, hipMemcpyDeviceToHost, sl.s));
        }
        CK(hipEventRecord(sl.done, sl.s));
        scatter(sp, sl.out.c(), sl.scatter);
        sl.busy = true;
    }
    for (size_t j = 0; j < (size_t)kSlots; ++j)
        RC(slot_retire(ctx, ctx->slots[(i + j) % kSlots]));
    for (Slot &sl : ctx->slots) {  // nothing in flight: the slabs go back to the process pool
        sl.in.release();
        sl.out.release();
    }
    return SEC_OK;
}

// ---- message batches (SHA-1 piece ids, bignum reduce, APDP tags) ------------
// `launch(base0, descs, n, out, stream)` runs the kernel over n messages whose
// descriptors are device-resident; out_per = output bytes per message.  Device
// mode: one launch over caller addresses.  SEC_F_HOST: messages are staged
// densely through pinned slabs (`slab` bytes) and the outputs copied back.
// `launch_kernel(base0, plan, sp, sub_index, out, stream)` runs the kernel(s) over the
// sub-plan's messages (descriptors device-resident at plan.meta + sp.off_msgs).
// seg_bytes > 0 also splits each message into segments of seg_bytes counted from its end
// (the least significant bytes of a big-endian integer) for the bignum reductions.
template <class Launch>
int msg_batch(sec_ctx *ctx, Plan &plan, const sec_msg *msgs, int64_t nmsgs, uint8_t *out, size_t out_per,
              unsigned flags, size_t slab, int kind, const char *what, uint64_t seg_bytes, Launch launch_kernel)
{
    // SHA-1 launches through kernels.hip, whose dispatches carry the timing events; the bignum
    // kernels (kind 3) are launched plainly, so their timing takes event records around them
    const bool attached = kind != 3;
    if (!ctx || nmsgs < 0 || (nmsgs > 0 && (!msgs || !out)) || (flags & ~(SEC_F_HOST | SEC_F_ASYNC)) ||
        nmsgs >= (int64_t)UINT32_MAX)
        return SEC_EINVAL;
    if (nmsgs == 0)
        return SEC_OK;
    const bool host = flags & SEC_F_HOST;
    RC(set_dev(ctx));
    std::vector<uint8_t> key;
    if (host) {  // dense staging: only lengths matter
        key.resize((size_t)nmsgs * 16);
        for (int64_t i = 0; i < nmsgs; ++i) {
            const uint64_t av = std::min(msgs[i].avail, msgs[i].len);
            memcpy(key.data() + i * 16, &msgs[i].len, 8);
            memcpy(key.data() + i * 16 + 8, &av, 8);
        }
    } else {
        key.assign((const uint8_t *)msgs, (const uint8_t *)(msgs + nmsgs));
    }
    const unsigned kflags = flags & ~SEC_F_ASYNC;  // ASYNC does not change the plan
    key.insert(key.end(), (const uint8_t *)&kflags, (const uint8_t *)&kflags + sizeof(unsigned));
    key.insert(key.end(), (const uint8_t *)&slab, (const uint8_t *)&slab + sizeof(size_t));
    key.insert(key.end(), (const uint8_t *)&seg_bytes, (const uint8_t *)&seg_bytes + sizeof(uint64_t));
    if (!(plan.valid && plan.key == key)) {
        plan.valid = false;
        std::vector<std::pair<int64_t, int64_t>> ranges;
        if (host) {
            std::vector<uint64_t> ib((size_t)nmsgs);
            for (int64_t i = 0; i < nmsgs; ++i)
                ib[i] = std::min(msgs[i].avail, msgs[i].len);
            ranges = slabs_of(ib, slab);
        } else {
            ranges.emplace_back(0, nmsgs);
        }
        Image img;
        plan.subs.clear();
        for (auto [c0, c1] : ranges) {
            SubPlan sp;
            sp.c0 = c0;
            sp.c1 = c1;
            sp.dig_first = (uint64_t)c0;
            std::vector<sec::MsgDesc> md;
            for (int64_t i = c0; i < c1; ++i) {
                const uint64_t av = std::min(msgs[i].avail, msgs[i].len);
                md.push_back(sec::MsgDesc{host ? sp.in_bytes : msgs[i].addr, msgs[i].len, av, 0, 0});
                sp.in_bytes += av;
            }
            sp.nmsgs = (uint32_t)md.size();
            sp.sha_split = sha1_split(ctx->opt, md);
            sp.out_bytes = (uint64_t)md.size() * out_per;
            sp.off_msgs = img.put(md.data(), md.size() * sizeof(sec::MsgDesc));
            if (seg_bytes) {
                std::vector<sec::SegDesc> segs;
                std::vector<sec::SegInfo> info;
                for (int64_t i = c0; i < c1; ++i) {
                    const uint64_t ns = std::max<uint64_t>(1, (msgs[i].len + seg_bytes - 1) / seg_bytes);
                    info.push_back(sec::SegInfo{(uint32_t)segs.size(), (uint32_t)ns});
                    for (uint64_t j = 0; j < ns; ++j)
                        segs.push_back(sec::SegDesc{(uint32_t)(i - c0), (uint32_t)j});
                    sp.max_seg = std::max<uint32_t>(sp.max_seg, (uint32_t)ns);
                }
                sp.nsegs = (uint32_t)segs.size();
                sp.off_segs = img.put(segs.data(), segs.size() * sizeof(sec::SegDesc));
                sp.off_seginfo = img.put(info.data(), info.size() * sizeof(sec::SegInfo));
            }
            plan.subs.push_back(std::move(sp));
        }
        std::vector<PendingExpand> none;
        RC(upload_plan(ctx, plan, img, ctx->enc_tabs, none));
        plan.key.swap(key);
        plan.valid = true;
    }
    if (!host) {
        const SubPlan &sp = plan.subs[0];
        hipEvent_t t0;
        RC(timing_begin(ctx, &t0, ctx->stream(), attached));
        int e = launch_kernel((const uint8_t *)nullptr, plan, sp, (size_t)0, out, ctx->stream());
        if (e)
            return hip_fail((hipError_t)e, what);
        RC(timing_end(ctx, t0, kind, ctx->stream()));
        if (!(flags & SEC_F_ASYNC))
            CK(hipStreamSynchronize(ctx->stream()));
        return SEC_OK;
    }
    auto gather = [&](const SubPlan &sp, char *stage, std::vector<sec::CopyJob> &jobs) {
        uint64_t o = 0;
        for (int64_t i = sp.c0; i < sp.c1; ++i) {
            const uint64_t av = std::min(msgs[i].avail, msgs[i].len);
            jobs.push_back(sec::CopyJob{stage + o, (const void *)(uintptr_t)msgs[i].addr, av});
            o += av;
        }
    };
    auto scatter = [&](const SubPlan &sp, char *stage, std::vector<sec::CopyJob> &jobs) {
        jobs.push_back(sec::CopyJob{out + sp.dig_first * out_per, stage, (size_t)sp.nmsgs * out_per});
    };
    auto launch = [&](const SubPlan &sp, uint8_t *din, uint8_t *dout, hipStream_t s) {
        hipEvent_t t0;
        RC(timing_begin(ctx, &t0, s, attached));
        int e = launch_kernel(din, plan, sp, (size_t)(&sp - plan.subs.data()), dout, s);
        if (e)
            return hip_fail((hipError_t)e, what);
        return timing_end(ctx, t0, kind, s);
    };
    return run_pipeline(ctx, plan, gather, scatter, launch);
}

// Runs `launch_kernel(dev_inputs[], dev_out, stream)` over `count` items whose inputs
// are dense arrays (sizes in `in_bytes`) and whose output is count * out_per bytes.
// SEC_F_HOST: inputs are uploaded into ctx->bn_scratch and the output copied back.
template <class Launch>
int dense_batch(sec_ctx *ctx, const std::vector<std::pair<const uint8_t *, size_t>> &ins, uint8_t *out,
                size_t out_bytes, unsigned flags, const char *what, Launch launch_kernel)
{
    RC(set_dev(ctx));
    const bool host = flags & SEC_F_HOST;
    hipStream_t s = ctx->stream();
    std::vector<const uint8_t *> dev;
    uint8_t *dout = out;
    if (host) {
        size_t tot = align_up(out_bytes, 256);
        for (auto &pr : ins)
            tot += align_up(pr.second, 256);
        RC(ctx->bn_scratch.ensure(tot));
        size_t o = 0;
        for (auto &pr : ins) {
            CK(hipMemcpyAsync(ctx->bn_scratch.as<uint8_t>(o), pr.first, pr.second, hipMemcpyHostToDevice, s));
            dev.push_back(ctx->bn_scratch.as<uint8_t>(o));
            o += align_up(pr.second, 256);
        }
        dout = ctx->bn_scratch.as<uint8_t>(o);
    } else {
        for (auto &pr : ins)
            dev.push_back(pr.first);
    }
    hipEvent_t t0;
    RC(timing_begin(ctx, &t0, s, false));
    int e = launch_kernel(dev, dout, s);
    if (e)
        return hip_fail((hipError_t)e, what);
    RC(timing_end(ctx, t0, 3, s));
    if (host)
        CK(hipMemcpyAsync(out, dout, out_bytes, hipMemcpyDeviceToHost, s));
    if (host || !(flags & SEC_F_ASYNC))
        CK(hipStreamSynchronize(s));
    return SEC_OK;
}

}  // namespace

// ============================================================================
extern "C" {

int sec_abi_version(void) { return SEC_ABI_VERSION; }

const char *sec_strerror(int s)
{
    switch (s) {
    case SEC_OK: return "ok";
    case SEC_EINVAL: return "invalid argument";
    case SEC_EKM: return "Precondition violation: 1 <= k <= m <= 256 required";
    case SEC_EBLOCKLEN: return "Precondition violation: Input blocks are required to be all the same length.";
    case SEC_ENBLOCKS: return "Precondition violation: exactly k blocks and k sharenums are required";
    case SEC_ESHARENUM: return "Precondition violation: sharenum is required to be in [0, m)";
    case SEC_EDUPSHARE: return "Precondition violation: duplicate sharenum";
    case SEC_EPADLEN: return "padlen larger than k * blocksize";
    case SEC_ESIZE: return "block size must be < 2^31 bytes";
    case SEC_ENODEV: return "no HIP device available";
    case SEC_EHIP: return "HIP runtime error";
    case SEC_ENOMEM: return "out of device or pinned memory";
    case SEC_ESINGULAR: return "decode matrix is singular";
    case SEC_EMODULUS: return "modulus must be an odd 2048-bit integer";
    case SEC_ENOTAG: return "key has no APDP tag constants (sec_bn_key_set_tag)";
    case SEC_ENOCRT: return "key has no CRT factors (sec_bn_key_set_crt)";
    default: return "unknown error";
    }
}

const char *sec_last_hip_error(void) { return g_hip_err.c_str(); }

int sec_device_count(int *count)
{
    if (!count)
        return SEC_EINVAL;
    *count = 0;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return SEC_ENODEV;
    *count = n;
    return SEC_OK;
}

int sec_ctx_create(int device, sec_ctx **out)
{
    if (!out)
        return SEC_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
        return SEC_ENODEV;
    sec_ctx *ctx = new sec_ctx();
    ctx->device = device;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess)
        // blocking w.r.t. the legacy NULL stream, so device buffers produced by work
        // there (e.g. torch's default stream) are ordered before our kernels and
        // results are ordered before the NULL stream's later work
        e = hipStreamCreateWithFlags(&ctx->own, hipStreamDefault);
    if (e == hipSuccess)
        e = hipEventCreateWithFlags(&ctx->pin_ev, hipEventDisableTiming);
    if (e == hipSuccess)
        e = hipEventCreateWithFlags(&ctx->meta_ev, hipEventDisableTiming);
    if (e == hipSuccess)
        e = hipEventRecord(ctx->pin_ev, ctx->own);
    if (e != hipSuccess) {
        sec_ctx_destroy(ctx);
        return hip_fail(e, "sec_ctx_create");
    }
    *out = ctx;
    return SEC_OK;
}

void sec_ctx_destroy(sec_ctx *ctx)
{
    if (!ctx)
        return;
    (void)hipSetDevice(ctx->device);
    (void)drain_all(ctx);
    if (ctx->own)
        (void)hipStreamSynchronize(ctx->own);
    for (auto &v : ctx->pending)
        for (auto &pr : v) {
            (void)hipEventDestroy(pr.first);
            (void)hipEventDestroy(pr.second);
        }
    for (auto e : ctx->ev_pool)
        (void)hipEventDestroy(e);
    if (ctx->pin_ev)
        (void)hipEventDestroy(ctx->pin_ev);
    if (ctx->meta_ev)
        (void)hipEventDestroy(ctx->meta_ev);
    for (Slot &s : ctx->slots) {
        s.in.release();
        s.out.release();
        s.din.release();
        s.dout.release();
        s.dsyn.release();
        if (s.done)
            (void)hipEventDestroy(s.done);
        if (s.s)
            (void)hipStreamDestroy(s.s);
    }
    ctx->tasks.reset();
    ctx->hash_tasks.reset();
    for (PinBuf &b : ctx->piece_par)
        b.release();
    ctx->pin.release();
    ctx->enc_tabs.buf.release();
    ctx->dec_tabs.buf.release();
    ctx->enc_plan.meta.release();
    ctx->dec_plan.meta.release();
    ctx->sha_plan.meta.release();
    ctx->bn_plan.meta.release();
    ctx->bn_scratch.release();
    ctx->bn_part.release();
    ctx->syn.release();
    if (ctx->own)
        (void)hipStreamDestroy(ctx->own);
    delete ctx;
}

int sec_ctx_set_stream(sec_ctx *ctx, void *stream)
{
    if (!ctx)
        return SEC_EINVAL;
    RC(set_dev(ctx));
    // order the switch: work queued so far completes before the new stream runs
    CK(hipStreamSynchronize(ctx->stream()));
    ctx->ext = (hipStream_t)stream;
    CK(hipEventRecord(ctx->pin_ev, ctx->stream()));
    return SEC_OK;
}

int sec_sync(sec_ctx *ctx)
{
    if (!ctx)
        return SEC_EINVAL;
    RC(set_dev(ctx));
    CK(hipStreamSynchronize(ctx->stream()));
    return SEC_OK;
}

int sec_ctx_set_timing(sec_ctx *ctx, int enable)
{
    if (!ctx)
        return SEC_EINVAL;
    ctx->timing = enable != 0;
    return SEC_OK;
}

int sec_ctx_set_option(sec_ctx *ctx, const char *name, int64_t value)
{
    const int i = opt_index(name);
    if (!ctx || i < 0)
        return SEC_EINVAL;
    if (value < kOpts[i].lo || value > kOpts[i].hi)
        return SEC_EINVAL;
    if (ctx->opt.v[i] == value)
        return SEC_OK;
    RC(set_dev(ctx));
    RC(drain_all(ctx));  // nothing in flight may still use a plan or pool built the old way
    ctx->opt.v[i] = value;
    for (Plan *p : {&ctx->enc_plan, &ctx->dec_plan, &ctx->sha_plan, &ctx->bn_plan})
        p->valid = false;
    if (i == O_COPY_THREADS) {
        ctx->tasks.reset();
        ctx->hash_tasks.reset();
    }
    return SEC_OK;
}

int sec_ctx_get_option(sec_ctx *ctx, const char *name, int64_t *value)
{
    const int i = opt_index(name);
    if (i < 0 || !value)
        return SEC_EINVAL;
    *value = ctx ? ctx->opt.v[i] : kOpts[i].dflt;  // NULL ctx: the default
    return SEC_OK;
}

const char *sec_option_name(int index)
{
    return index >= 0 && index < O_COUNT ? kOpts[index].name : nullptr;
}

int sec_timing_collect(sec_ctx *ctx, int kind, double *total_ms, int64_t *launches)
{
    if (!ctx || kind < 0 || kind > 3 || !total_ms || !launches)
        return SEC_EINVAL;
    RC(set_dev(ctx));
    double tot = 0;
    for (auto &pr : ctx->pending[kind]) {
        CK(hipEventSynchronize(pr.second));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, pr.first, pr.second));
        tot += ms;
        ctx->ev_pool.push_back(pr.first);
        ctx->ev_pool.push_back(pr.second);
    }
    *launches = (int64_t)ctx->pending[kind].size();
    *total_ms = tot;
    ctx->pending[kind].clear();
    return SEC_OK;
}

// Which k of the n blocks a caller holds to decode from (storb's validator fetches every data and
// parity piece of a chunk, /root/reference/storb/validator/validator.py:1556-1604, 1631; the
// reference then takes the first k in piece order, storb/util/piece.py:189-191).  Any k distinct
// blocks give the same bytes, so the choice is free, and it decides the decode's cost:
//   * every present primary (its bytes are copied, not computed);
//   * the e = k - primaries parity rows from as few bit-sliced row groups as possible
//     (sec_bs_rows(sec_syn_shape(k, m)) rows each: 16 for the policy's wide shapes): one group
//     holding e present rows lets an e <= 16 decode take the fused one-wave syndrome kernel
//     (api.cpp syn_choice), where rows spread over both groups of zfec(64,96) read the data once
//     per group; groups with the most present rows first, lowest rows first within a group.
// Entries that are out of range or repeat an earlier sharenum are never chosen.  pick[0..k) =
// positions in `sharenums`, in ascending sharenum order.  SEC_ENBLOCKS when fewer than k
// distinct valid blocks are present.
int sec_decode_choose(int k, int m, int64_t n, const int32_t *sharenums, int32_t *pick)
{
    if (!pick || n < 0 || (n > 0 && !sharenums))
        return SEC_EINVAL;
    if (k < 1 || m < k || m > 256)
        return SEC_EKM;
    int pos[256];
    for (int j = 0; j < 256; ++j)
        pos[j] = -1;
    int distinct = 0;
    for (int64_t i = 0; i < n; ++i) {
        const int s = sharenums[i];
        if (s >= 0 && s < m && pos[s] < 0) {
            pos[s] = (int)i;
            ++distinct;
        }
    }
    if (distinct < k)
        return SEC_ENBLOCKS;
    bool take[256] = {false};
    int have = 0;
    for (int j = 0; j < k; ++j)
        if (pos[j] >= 0) {
            take[j] = true;
            ++have;
        }
    const int e = k - have, p = m - k;
    if (e > 0) {
        const int sh = sec_syn_shape(k, m);
        const int G = sh >= 0 ? sec_bs_rows(sh) : p;
        const int ng = (p + G - 1) / G;
        std::vector<int> cnt((size_t)ng, 0);
        for (int r = 0; r < p; ++r)
            cnt[(size_t)(r / G)] += pos[k + r] >= 0;
        std::vector<int> order((size_t)ng);
        for (int g = 0; g < ng; ++g)
            order[(size_t)g] = g;
        int one = -1;  // lowest group that alone holds e present rows
        for (int g = 0; g < ng && one < 0; ++g)
            if (cnt[(size_t)g] >= e)
                one = g;
        if (one >= 0)
            order = {one};
        else
            std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return cnt[(size_t)a] > cnt[(size_t)b]; });
        int need = e;
        for (int g : order)
            for (int r = g * G; r < std::min(p, (g + 1) * G) && need > 0; ++r)
                if (pos[k + r] >= 0) {
                    take[k + r] = true;
                    --need;
                }
    }
    int o = 0;
    for (int j = 0; j < m; ++j)
        if (take[j])
            pick[o++] = pos[j];
    return SEC_OK;
}

int sec_encode_matrix(int k, int m, uint8_t *out)
{
    if (!out)
        return SEC_EINVAL;
    if (k < 1 || m < k || m > 256)
        return SEC_EKM;
    const std::vector<uint8_t> enc = sec::encode_matrix(k, m);
    memcpy(out, enc.data() + (size_t)k * k, (size_t)(m - k) * k);
    return SEC_OK;
}

int sec_decode_matrix(int k, int m, const int32_t *sharenums, uint8_t *out, int32_t *out_index)
{
    if (!sharenums || !out)
        return SEC_EINVAL;
    if (k < 1 || m < k || m > 256)
        return SEC_EKM;
    RC(check_sharenums(k, m, sharenums));
    std::vector<int> idx(sharenums, sharenums + k), perm;
    sec::normalise_slots(k, idx, perm);
    std::vector<uint8_t> minv;
    if (!sec::decode_matrix(k, m, idx, minv))
        return SEC_ESINGULAR;
    memcpy(out, minv.data(), (size_t)k * k);
    if (out_index)
        for (int i = 0; i < k; ++i)
            out_index[i] = idx[i];
    return SEC_OK;
}

// ---------------------------------------------------------------------------
}  // extern "C"

namespace {

// The caller byte ranges [a, a + len) a host call reads or writes.
struct HostRange {
    uintptr_t a;
    uint64_t len;
    bool out = false;  // the kernels write it (a decode's output, an encode's parity)
};

std::vector<HostRange> encode_ranges(const sec_enc_chunk *chunks, int64_t nchunks, const uint8_t *in,
                                     const uint8_t *parity)
{
    std::vector<HostRange> r;
    for (int64_t i = 0; i < nchunks; ++i) {
        const sec_enc_chunk &c = chunks[i];
        const uint64_t B = (c.n + (uint64_t)c.k - 1) / (uint64_t)c.k, p = (uint64_t)(c.m - c.k);
        r.push_back(HostRange{(uintptr_t)in + c.in_off, c.n});
        if (p && B)
            r.push_back(HostRange{(uintptr_t)parity + c.parity_off, (p - 1) * c.parity_stride + B, true});
    }
    return r;
}

std::vector<HostRange> decode_ranges(const sec_dec_chunk *chunks, int64_t nchunks, const int32_t *sharenums,
                                     const uint64_t *block_offs, const uint64_t *block_avail, const uint8_t *blocks,
                                     const uint8_t *out, bool recover)
{
    std::vector<HostRange> r;
    for (int64_t i = 0; i < nchunks; ++i) {
        const sec_dec_chunk &c = chunks[i];
        r.push_back(HostRange{(uintptr_t)out + c.out_off, dec_nout(c, sharenums, recover), true});
        for (int j = 0; j < c.k; ++j)
            r.push_back(HostRange{(uintptr_t)blocks + block_offs[c.slot0 + j], slot_avail(c, block_avail, j)});
    }
    return r;
}

// Pages host calls lock for themselves (transient registrations), process-wide.  A call's
// HostLock page-locks pageable caller buffers (hipHostRegister) for the call's duration so the
// kernels can run on them directly; ranges less than 4 MiB apart are locked as one, so a
// registration can cover memory of other callers too.  Such pages must never count as pinned
// for any other call: its owner unlocks them when its own stream has drained, whatever the
// other call's kernels are doing, and memory freed and reused inside a registration would map
// to the old pages on the device.  So every transient registration is recorded here, and a
// range that touches one is never zero-copy for a call that does not hold it (that call is
// staged).  Classification and locking happen under one mutex.
struct TransientLocks {
    std::mutex mu;
    std::map<uintptr_t, uintptr_t> regs;  // page-aligned [lo, hi) of every transient registration

    // true when [a, a + len) overlaps a registration
    bool touches(uintptr_t a, uint64_t len) const
    {
        auto it = regs.upper_bound(a);  // first registration starting after a
        if (it != regs.begin() && std::prev(it)->second > a)
            return true;
        return it != regs.end() && it->first < a + len;
    }
};

TransientLocks &transient_locks()
{
    static TransientLocks t;
    return t;
}

// Locking is used when the call moves at least SEC_REGISTER_MIN bytes (default 4 MiB; 0 =
// never) in ranges of 1 MiB or more on average once ranges less than 4 MiB apart are merged
// (one registration per small, separate buffer would cost more than copying it).  Locking
// 1 GiB took 2.1 ms and unlocking 0.05 ms (tools/e2e_study.py), against tens of ms for the
// two staging copies.  Any failure (memory registered elsewhere, unregistrable mappings)
// releases what was locked and the call is staged.  Released on every return path, after
// the call's stream has drained.
class HostLock {
public:
    explicit HostLock(hipStream_t s) : s_(s) {}
    ~HostLock() { release(); }
    HostLock(const HostLock &) = delete;
    HostLock &operator=(const HostLock &) = delete;

    // 0: staged; 1: every range in persistently pinned memory (zero-copy, nothing locked);
    // 2: zero-copy on pages this call locked (plus persistently pinned ones).  dry: lock
    // nothing, 2 = the ranges pass the size rules (a lock would be tried)
    int acquire(const std::vector<HostRange> &rs, int64_t register_min, bool may_lock = true, bool dry = false)
    {
        TransientLocks &tl = transient_locks();
        std::lock_guard<std::mutex> g(tl.mu);
        uint64_t total = 0;
        std::vector<std::pair<uintptr_t, uintptr_t>> pg;  // page-aligned [lo, hi) of pageable ranges
        PinnedRange cache;
        for (const HostRange &r : rs) {
            if (!r.len)
                continue;
            total += r.len;
            if (tl.touches(r.a, r.len))
                return 0;  // another call's transient pages: neither pinned nor lockable for us
            if (!pinned(r.a, r.len, &cache))  // persistently pinned (sec_host_alloc / _register)
                pg.emplace_back(r.a & ~kPageMask, (r.a + r.len + kPageMask) & ~kPageMask);
        }
        if (pg.empty())
            return 1;
        if (!may_lock || register_min <= 0 || total < (uint64_t)register_min)
            return 0;
        std::sort(pg.begin(), pg.end());
        // ranges less than kGap apart are locked as one (e.g. around a decode's erased blocks);
        // if that swallows memory that cannot be locked, retry with exact ranges once
        for (const uintptr_t gap : {kGap, (uintptr_t)0}) {
            std::vector<std::pair<uintptr_t, uintptr_t>> merged;
            for (auto &q : pg)
                if (!merged.empty() && q.first <= merged.back().second + gap)
                    merged.back().second = std::max(merged.back().second, q.second);
                else
                    merged.push_back(q);
            if (merged.size() * ((uint64_t)1 << 20) > total)
                return 0;
            if (dry)
                return 2;
            for (const HostRange &r : rs)
                if (r.out && r.len && !pinned(r.a, r.len, &cache))
                    fault_in(r.a, r.len);
            bool ok = true;
            for (auto &q : merged) {
                if (tl.touches(q.first, q.second - q.first) ||
                    hipHostRegister((void *)q.first, q.second - q.first, hipHostRegisterDefault) != hipSuccess) {
                    (void)hipGetLastError();
                    ok = false;
                    break;
                }
                locked_.push_back(q);
                tl.regs.emplace(q.first, q.second);
            }
            if (ok) {
                // the runtime must map what it locked at the same address on the device
                PinnedRange c2;
                for (const HostRange &r : rs)
                    if (r.len && !pinned(r.a, r.len, &c2))
                        ok = false;
                if (ok)
                    return 2;
            }
            unlock_all(tl);
        }
        return 0;
    }

    void release()
    {
        if (locked_.empty())
            return;
        (void)hipStreamSynchronize(s_);  // nothing of this call may still run on the pages
        TransientLocks &tl = transient_locks();
        std::lock_guard<std::mutex> g(tl.mu);
        unlock_all(tl);
    }

private:
    static constexpr uintptr_t kPageMask = 4095;

    // Every page of [a, a + len) the kernels will write and the process has not touched yet
    // (mincore: not resident) is faulted in writable by the CPU first, by an atomic OR of 0 into
    // one byte of the range on that page (no value changes, and no store of another thread to
    // that byte can be lost), so no output page is unbacked when the device maps it.  Round 6
    // saw one wrong reassembled row whose output pages the host had never touched (DESIGN §5
    // Round 6).  Resident pages cost nothing but the one mincore call.
    static void fault_in(uintptr_t a, uint64_t len)
    {
        const uintptr_t lo = a & ~kPageMask, hi = (a + len + kPageMask) & ~kPageMask;
        const size_t np = (hi - lo) >> 12;
        std::vector<unsigned char> res(np, 0);
        const bool known = mincore((void *)lo, hi - lo, res.data()) == 0;
        for (size_t i = 0; i < np; ++i)
            if (!known || !(res[i] & 1)) {
                const uintptr_t b = std::max<uintptr_t>(a, lo + (i << 12));
                (void)__atomic_fetch_or((uint8_t *)b, (uint8_t)0, __ATOMIC_RELAXED);
            }
    }
    static constexpr uintptr_t kGap = (uintptr_t)4 << 20;
    void unlock_all(TransientLocks &tl)  // tl.mu held
    {
        for (auto &q : locked_) {
            (void)hipHostUnregister((void *)q.first);
            tl.regs.erase(q.first);
        }
        (void)hipGetLastError();
        locked_.clear();
    }
    hipStream_t s_;
    std::vector<std::pair<uintptr_t, uintptr_t>> locked_;
};

// Decides a host call's path: zero-copy on the caller's pinned buffers, zero-copy on pages
// locked for the call (`lock`), or staged.  True = run the device path on host addresses.
bool host_direct(sec_ctx *ctx, const std::vector<HostRange> &rs, HostLock &lock, unsigned flags)
{
    switch (lock.acquire(rs, ctx->opt[O_REGISTER_MIN], !(flags & SEC_F_STAGED))) {
    case 1: ++ctx->zero_copy_calls; return true;
    case 2: ++ctx->registered_calls; return true;
    default: ++ctx->staged_calls; return false;
    }
}

// sec_encode_batch (digests == nullptr, digest == false) and sec_encode_digest_batch.
int encode_impl(sec_ctx *ctx, const sec_enc_chunk *chunks, int64_t nchunks, const uint8_t *in, uint8_t *parity,
                uint8_t *digests, unsigned flags, int digest)
{
    if (!ctx || nchunks < 0 || (nchunks > 0 && !chunks) || (flags & ~(SEC_F_HOST | SEC_F_ASYNC | SEC_F_STAGED)) ||
        ((flags & SEC_F_STAGED) && !(flags & SEC_F_HOST)))
        return SEC_EINVAL;
    if (nchunks == 0)
        return SEC_OK;
    if (nchunks >= (int64_t)UINT32_MAX)
        return SEC_EINVAL;
    bool host = flags & SEC_F_HOST;
    RC(set_dev(ctx));

    // easyfec.Encoder.encode / _fec.Encoder preconditions
    uint64_t total_par = 0, total_in = 0;
    for (int64_t i = 0; i < nchunks; ++i) {
        const sec_enc_chunk &c = chunks[i];
        if (c.k < 1 || c.m < c.k || c.m > 256)
            return SEC_EKM;
        const uint64_t B = enc_B(c);
        if (c.k > 1 && (uint64_t)(c.k - 1) * B > c.n)
            return SEC_EBLOCKLEN;
        if (B >= (1ull << 31))
            return SEC_ESIZE;
        const uint64_t p = (uint64_t)(c.m - c.k);
        if (p > 0 && B > 0 && c.parity_stride < B)
            return SEC_EINVAL;
        total_par += p * B;
        total_in += c.n;
    }
    if (total_par == 0 && !digest)
        return SEC_OK;  // nothing to compute (m == k, or empty chunks)
    if ((!in && !host && total_in) || (!parity && total_par) || (digest && !digests))
        return SEC_EINVAL;
    // pinned (or lockable) caller buffers: run the device path on them directly (synchronous,
    // as every host call).  Digest mode keeps the staged path: SHA-1 is one latency-bound lane
    // per piece, which would stall on every PCIe read.
    HostLock lock(ctx->stream());
    if (host && !digest && host_direct(ctx, encode_ranges(chunks, nchunks, in, parity), lock, flags)) {
        host = false;
        flags &= ~(SEC_F_HOST | SEC_F_ASYNC);
    } else if (host && digest) {
        ++ctx->staged_calls;  // (host_direct counted the other staged calls)
    }

    // Plan key: the whole descriptor array for device mode; only the shapes for
    // host mode (its device layout is dense, caller addresses are used by the
    // gather / scatter alone), so repeated per-chunk calls reuse one plan.
    Plan &plan = ctx->enc_plan;
    std::vector<uint8_t> key;
    if (host) {
        key.resize((size_t)nchunks * 16);
        for (int64_t i = 0; i < nchunks; ++i) {
            memcpy(key.data() + i * 16, &chunks[i].n, 8);
            memcpy(key.data() + i * 16 + 8, &chunks[i].k, 4);
            memcpy(key.data() + i * 16 + 12, &chunks[i].m, 4);
        }
    } else {
        key.resize(sizeof(sec_enc_chunk) * (size_t)nchunks);
        memcpy(key.data(), chunks, sizeof(sec_enc_chunk) * (size_t)nchunks);
    }
    // ASYNC and STAGED do not change the plan
    const unsigned kflags = (flags & ~(SEC_F_ASYNC | SEC_F_STAGED)) | ((unsigned)digest << 16);
    key.insert(key.end(), (const uint8_t *)&kflags, (const uint8_t *)&kflags + sizeof(unsigned));
    if (!(plan.valid && plan.gen == ctx->enc_tabs.gen && plan.key == key)) {
        plan.valid = false;
        RC(build_encode_plan(ctx, chunks, nchunks, host, digest));
        plan.key.swap(key);
        plan.valid = true;
    }

    if (!host) {
        hipEvent_t t0 = nullptr;
        RC(timing_begin(ctx, &t0, ctx->stream()));
        RC(launch_encode_sub(ctx, plan, plan.subs[0], in, parity, digests, ctx->stream()));
        RC(timing_end(ctx, t0, 0, ctx->stream()));
        if (!(flags & SEC_F_ASYNC))
            CK(hipStreamSynchronize(ctx->stream()));
        return SEC_OK;
    }
    auto gather = [&](const SubPlan &sp, char *stage, std::vector<sec::CopyJob> &jobs) {
        uint64_t o = 0;
        for (int64_t i = sp.c0; i < sp.c1; ++i) {
            jobs.push_back(sec::CopyJob{stage + o, in + chunks[i].in_off, chunks[i].n});
            o += chunks[i].n;
        }
    };
    auto scatter = [&](const SubPlan &sp, char *stage, std::vector<sec::CopyJob> &jobs) {
        uint64_t o = 0;
        for (int64_t i = sp.c0; i < sp.c1; ++i) {
            const sec_enc_chunk &c = chunks[i];
            const uint64_t B = enc_B(c), p = (uint64_t)(c.m - c.k);
            if (c.parity_stride == B) {
                jobs.push_back(sec::CopyJob{parity + c.parity_off, stage + o, p * B});
            } else {
                for (uint64_t r = 0; r < p; ++r)
                    jobs.push_back(sec::CopyJob{parity + c.parity_off + r * c.parity_stride, stage + o + r * B, B});
            }
            o += p * B;
        }
        if (sp.nmsgs)
            jobs.push_back(sec::CopyJob{digests + sp.dig_first * 20, stage + sp.dig_off, (size_t)sp.nmsgs * 20});
    };
    auto launch = [&](const SubPlan &sp, uint8_t *din, uint8_t *dout, hipStream_t s) {
        return launch_encode_sub(ctx, plan, sp, din, dout, dout + sp.dig_off, s);
    };
    return run_pipeline(ctx, plan, gather, scatter, launch, !digest);
}

}  // namespace

extern "C" {

int sec_encode_batch(sec_ctx *ctx, const sec_enc_chunk *chunks, int64_t nchunks, const uint8_t *in,
                     uint8_t *parity, unsigned flags)
{
    return encode_impl(ctx, chunks, nchunks, in, parity, nullptr, flags, 0);
}

int sec_encode_digest_batch(sec_ctx *ctx, const sec_enc_chunk *chunks, int64_t nchunks, const uint8_t *in,
                            uint8_t *parity, uint8_t *digests, unsigned flags)
{
    return encode_impl(ctx, chunks, nchunks, in, parity, digests, flags, 1);
}

// easyfec's Encoder.encode output for every chunk, as pieces in caller buffers: the k data
// slices (copies, the last zero-padded to B) and the m - k parity blocks, each in its own buffer,
// plus (digests) each piece's SHA-1.  The data pieces are copied and hashed on the context's
// task threads while this thread runs the encode (the parity into a pinned scratch); the parity
// pieces are copied and hashed as soon as it returns.  Everything but the GPU call is host work
// that the Python layer would otherwise do on its own threads, under the GIL's hand-offs
// (VERDICT r04 next #7).
int sec_encode_pieces(sec_ctx *ctx, const sec_enc_chunk *chunks, int64_t nchunks, const uint8_t *in,
                      uint8_t *const *pieces, uint8_t *digests, unsigned flags)
{
    if (!ctx || nchunks < 0 || (nchunks > 0 && (!chunks || !pieces)) || !(flags & SEC_F_HOST) ||
        (flags & ~(SEC_F_HOST | SEC_F_STAGED | SEC_F_GPU_PARITY_IDS)))
        return SEC_EINVAL;
    // parity ids on the GPU: only with digests (else the flag changes nothing)
    const bool gpu_ids = digests && (flags & SEC_F_GPU_PARITY_IDS);
    if (nchunks == 0)
        return SEC_OK;
    if (nchunks >= (int64_t)UINT32_MAX)
        return SEC_EINVAL;
    uint64_t max_par = 0;
    for (int64_t i = 0; i < nchunks; ++i) {  // easyfec / _fec preconditions (as encode_impl)
        const sec_enc_chunk &c = chunks[i];
        if (c.k < 1 || c.m < c.k || c.m > 256)
            return SEC_EKM;
        const uint64_t B = enc_B(c);
        if (c.k > 1 && (uint64_t)(c.k - 1) * B > c.n)
            return SEC_EBLOCKLEN;
        if (B >= (1ull << 31))
            return SEC_ESIZE;
        max_par = std::max<uint64_t>(max_par, (uint64_t)(c.m - c.k) * B);
    }
    for (int64_t i = 0, pb = 0; i < nchunks; pb += chunks[i++].m)  // a buffer for every non-empty piece
        for (int j = 0; j < chunks[i].m; ++j)
            if (!pieces[pb + j] && enc_B(chunks[i]) > 0)
                return SEC_EINVAL;
    RC(set_dev(ctx));
    // The parity goes through pinned scratch in sub-batches of at most `cap` bytes (a chunk whose
    // own parity is larger alone), two scratch buffers in turn: sub-batch s + 1 encodes while the
    // task threads copy and hash sub-batch s's parity pieces.  Locked memory stays bounded by
    // 2 cap whatever the call's size (one allocation of the whole call's parity).
    // With gpu_ids the GPU hashes a sub-batch's parity pieces in one chain time (one lane per
    // piece), so the sub-batches are SEC_SLAB_BYTES_DIGEST: as many pieces in flight as it allows.
    const uint64_t cap =
        std::max<uint64_t>((uint64_t)ctx->opt[gpu_ids ? O_SLAB_BYTES_DIGEST : O_SLAB_BYTES], max_par);
    std::vector<uint8_t> par_dig;  // gpu_ids: a sub-batch's parity digests, chunk by chunk
    sec::TaskPool &tp = hash_tasks(ctx);
    sec::TaskPool::Group data, par[2];
    bool par_failed = false;
    std::vector<sec_enc_chunk> tmp(chunks, chunks + nchunks);
    std::vector<uint64_t> first_piece((size_t)nchunks);
    uint64_t pb = 0;
    for (int64_t i = 0; i < nchunks; ++i) {
        const sec_enc_chunk &c = chunks[i];
        const uint64_t B = enc_B(c);
        first_piece[i] = pb;
        for (int j = 0; j < c.m && B == 0; ++j)  // an empty chunk: every piece is b"" (no buffer)
            if (digests)
                (void)sec::sha1_padded(nullptr, 0, 0, digests + (pb + j) * 20);
        for (int j = 0; j < c.k && B > 0; ++j) {
            const uint64_t start = (uint64_t)j * B;
            const uint64_t av = c.n > start ? std::min<uint64_t>(B, c.n - start) : 0;
            uint8_t *dst = pieces[pb + j];
            // (a NULL `in` with absolute in_off is legal here, as in sec_encode_batch's host mode)
            const uint8_t *src = (const uint8_t *)((uintptr_t)in + c.in_off + start);
            uint8_t *dig = digests ? digests + (pb + j) * 20 : nullptr;
            tp.submit(data, [=] {
                if (av)
                    memcpy(dst, src, av);
                if (av < B)
                    memset(dst + av, 0, B - av);
                return !dig || sec::sha1_padded(dst, B, B, dig);
            });
        }
        pb += (uint64_t)c.m;
    }
    int rc = SEC_OK;
    int buf = 0;
    for (int64_t c0 = 0; c0 < nchunks && rc == SEC_OK;) {
        // the next sub-batch [c0, c1): chunks whose parity sums to at most cap
        int64_t c1 = c0;
        uint64_t po = 0;
        while (c1 < nchunks) {
            const sec_enc_chunk &c = chunks[c1];
            const uint64_t B = enc_B(c), p = (uint64_t)(c.m - c.k) * B;
            if (c1 > c0 && po + p > cap)
                break;
            tmp[c1].parity_off = po;
            tmp[c1].parity_stride = B;
            po += p;
            ++c1;
        }
        if (po) {
            par_failed |= !tp.wait(par[buf]);  // the scratch's previous pieces are copied out
            par[buf].failed.store(false);
            PinBuf &scratch = ctx->piece_par[buf];
            rc = scratch.ensure(po);
            if (rc == SEC_OK && gpu_ids) {
                // parity and its ids in one staged call: the SHA-1 kernel runs on the device
                // parity right after the encode (slots: each chunk's m - k, in chunk order)
                uint64_t np = 0;
                for (int64_t i = c0; i < c1; ++i)
                    np += (uint64_t)(chunks[i].m - chunks[i].k);
                try {
                    par_dig.resize((size_t)np * 20);
                } catch (const std::bad_alloc &) {
                    rc = SEC_ENOMEM;
                }
                if (rc == SEC_OK)
                    rc = encode_impl(ctx, tmp.data() + c0, c1 - c0, in, (uint8_t *)scratch.p, par_dig.data(),
                                     SEC_F_HOST | (flags & SEC_F_STAGED), 2);
                for (int64_t i = c0, q = 0; i < c1 && rc == SEC_OK; ++i)
                    for (int r = 0; r < chunks[i].m - chunks[i].k; ++r, ++q)
                        if (enc_B(chunks[i]) > 0)  // (an empty chunk's ids are sha1(b"") from above)
                            memcpy(digests + (first_piece[i] + chunks[i].k + r) * 20, par_dig.data() + q * 20, 20);
            } else if (rc == SEC_OK) {
                rc = encode_impl(ctx, tmp.data() + c0, c1 - c0, in, (uint8_t *)scratch.p, nullptr,
                                 SEC_F_HOST | (flags & SEC_F_STAGED), 0);
            }
            for (int64_t i = c0; i < c1 && rc == SEC_OK; ++i) {
                const sec_enc_chunk &c = chunks[i];
                const uint64_t B = enc_B(c);
                for (int r = 0; r < c.m - c.k && B > 0; ++r) {
                    uint8_t *dst = pieces[first_piece[i] + c.k + r];
                    const uint8_t *src = (const uint8_t *)scratch.p + tmp[i].parity_off + (uint64_t)r * B;
                    uint8_t *dig = digests && !gpu_ids ? digests + (first_piece[i] + c.k + r) * 20 : nullptr;
                    tp.submit(par[buf], [=] {
                        memcpy(dst, src, B);
                        return !dig || sec::sha1_padded(dst, B, B, dig);
                    });
                }
            }
            buf ^= 1;
        }
        c0 = c1;
    }
    // every group waited: no task outlives the call
    const bool ok_data = tp.wait(data);
    for (sec::TaskPool::Group &g : par)
        par_failed |= !tp.wait(g);
    if (rc == SEC_OK && (!ok_data || par_failed))
        rc = SEC_EINVAL;  // OpenSSL failed (no other cause)
    for (PinBuf &b : ctx->piece_par)  // every task waited: the scratch goes back to the process pool
        b.release();
    return rc;
}

int sec_sha1_batch(sec_ctx *ctx, const sec_msg *msgs, int64_t nmsgs, uint8_t *digests, unsigned flags)
{
    if (!ctx)
        return SEC_EINVAL;
    return msg_batch(ctx, ctx->sha_plan, msgs, nmsgs, digests, 20, flags,
                     (size_t)ctx->opt[O_SLAB_BYTES_DIGEST], 2, "sec_sha1_kernel", 0,
                     [](const uint8_t *base0, const Plan &plan, const SubPlan &sp, size_t, uint8_t *o, hipStream_t s) {
                         return sec_launch_sha1(base0, nullptr, plan.meta.as<sec::MsgDesc>(sp.off_msgs), sp.nmsgs, o,
                                                s, sp.sha_split);
                     });
}

// ---------------------------------------------------------------------------
// APDP bignum (bignum.hip).  The key lives on the device of the context that
// created it: a TagKey whose first member is the BnKey.
}  // extern "C"

struct sec_bn_key {
    int device = 0;
    DevBuf dk;     // TagKey, then 1 KiB of upload staging
    DevBuf table;  // fixed-base table of g (sec::kGTabWords u32), once set_tag ran
    bool has_tag = false, has_crt = false;
    mutable DevBuf rpow;              // R^(j S) mod n (Montgomery form), j < rpow_count
    mutable uint32_t rpow_count = 0;  // grown on demand by the segmented reductions
};

namespace {
constexpr size_t kKeyStage = sizeof(sec::TagKey);

uint32_t neg_inv32(const uint8_t *be, size_t nbytes)  // -n^-1 mod 2^32 from n's low limb
{
    const uint8_t *p = be + nbytes - 4;
    const uint32_t n0 = (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
    uint32_t x = n0;  // n0 * n0 == 1 mod 8: 3 correct bits, doubling per Newton step
    for (int i = 0; i < 4; ++i)
        x *= 2u - n0 * x;
    return 0u - x;
}

bool odd_top(const uint8_t *be, size_t nbytes) { return (be[0] & 0x80) && (be[nbytes - 1] & 1); }

// Segmented reductions: every message is cut into kSegBytes segments from its end, one
// wave each (so a batch of few, large pieces still fills the chip); partial residues
// r_j * R^(j S) go to ctx->bn_part, then one wave per message sums them.
constexpr uint64_t kSegBytes = (uint64_t)sec::kSegChunks * 256;

int bn_prepare(sec_ctx *ctx, const sec_bn_key *key, const Plan &plan, bool host)
{
    uint32_t need = 0;
    size_t part = 0;
    for (const SubPlan &sp : plan.subs) {
        need = std::max(need, sp.max_seg);
        part = std::max(part, (size_t)sp.nsegs * 256);
    }
    if (need > key->rpow_count) {  // grow R^(j S) to cover the longest message
        const uint32_t cap = std::max<uint32_t>(need, 2 * key->rpow_count);
        DevBuf grown;
        RC(grown.ensure((size_t)cap * 256));
        if (key->rpow_count)
            CK(hipMemcpyAsync(grown.p, key->rpow.p, (size_t)key->rpow_count * 256, hipMemcpyDeviceToDevice,
                              ctx->stream()));
        int e = sec_launch_bn_rpow(key->dk.as<sec::BnKey>(), key->rpow_count, cap, grown.as<uint32_t>(), ctx->stream());
        if (e)
            return hip_fail((hipError_t)e, "sec_bn_rpow_kernel");
        CK(hipStreamSynchronize(ctx->stream()));
        key->rpow.release();
        key->rpow = grown;
        grown.p = nullptr;
        key->rpow_count = cap;
    }
    ctx->bn_part_stride = part;
    return ctx->bn_part.ensure(std::max<size_t>(part, 256) * (host ? kSlots : 1));
}

uint8_t *bn_part(sec_ctx *ctx, size_t sub_index, bool host)
{
    return ctx->bn_part.as<uint8_t>(host ? (sub_index % kSlots) * ctx->bn_part_stride : 0);
}
}  // namespace

extern "C" {

int sec_bn_key_create(sec_ctx *ctx, const uint8_t *n_be, sec_bn_key **out)
{
    if (!ctx || !n_be || !out)
        return SEC_EINVAL;
    *out = nullptr;
    if (!odd_top(n_be, 256))
        return SEC_EMODULUS;
    RC(set_dev(ctx));
    std::unique_ptr<sec_bn_key> key(new sec_bn_key());
    key->device = ctx->device;
    RC(key->dk.ensure(kKeyStage + 1024));
    CK(hipMemsetAsync(key->dk.p, 0, sizeof(sec::TagKey), ctx->stream()));
    uint8_t *nd = key->dk.as<uint8_t>(kKeyStage);
    hipStream_t s = ctx->stream();
    CK(hipMemcpyAsync(nd, n_be, 256, hipMemcpyHostToDevice, s));
    int e = sec_launch_bn_setup(nd, neg_inv32(n_be, 256), 2048, key->dk.as<sec::BnKey>(), s);
    if (e)
        return hip_fail((hipError_t)e, "sec_bn_setup_kernel");
    CK(hipStreamSynchronize(s));
    *out = key.release();
    return SEC_OK;
}

void sec_bn_key_destroy(sec_bn_key *key)
{
    if (!key)
        return;
    (void)hipSetDevice(key->device);
    key->dk.release();
    key->table.release();
    key->rpow.release();
    delete key;
}

int sec_bn_key_set_crt(sec_ctx *ctx, sec_bn_key *key, const uint8_t *p_be, const uint8_t *q_be, const uint8_t *cp_be,
                       const uint8_t *cq_be)
{
    if (!ctx || !key || !p_be || !q_be || !cp_be || !cq_be || key->device != ctx->device)
        return SEC_EINVAL;
    if (!odd_top(p_be, 128) || !odd_top(q_be, 128))
        return SEC_EMODULUS;
    RC(set_dev(ctx));
    uint8_t host[768];
    memcpy(host, p_be, 128);
    memcpy(host + 128, q_be, 128);
    memcpy(host + 256, cp_be, 256);
    memcpy(host + 512, cq_be, 256);
    uint8_t *st = key->dk.as<uint8_t>(kKeyStage);
    sec::TagKey *tk = key->dk.as<sec::TagKey>();
    hipStream_t s = ctx->stream();
    CK(hipMemcpyAsync(st, host, sizeof(host), hipMemcpyHostToDevice, s));
    int e = sec_launch_bn_setup(st, neg_inv32(p_be, 128), 1024, &tk->p, s);
    if (!e)
        e = sec_launch_bn_setup(st + 128, neg_inv32(q_be, 128), 1024, &tk->q, s);
    if (!e)
        e = sec_launch_crt_setup(st + 256, st + 512, tk, s);
    if (e)
        return hip_fail((hipError_t)e, "sec_bn_key_set_crt");
    const uint32_t off = 0;  // tags need dp / dq too: CRT tags switch on in set_tag
    CK(hipMemcpyAsync(&tk->crt, &off, sizeof(off), hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    key->has_crt = true;
    return SEC_OK;
}

int sec_bn_key_set_tag(sec_ctx *ctx, sec_bn_key *key, const uint8_t *g_be, const uint8_t *fdh_be,
                       const uint8_t *d_be, const uint8_t *dp_be, const uint8_t *dq_be)
{
    if (!ctx || !key || !g_be || !fdh_be || !d_be || key->device != ctx->device || (!dp_be != !dq_be))
        return SEC_EINVAL;
    const bool crt = dp_be != nullptr;
    if (crt && !key->has_crt)
        return SEC_ENOCRT;
    RC(set_dev(ctx));
    uint8_t host[1024] = {0};
    memcpy(host, g_be, 256);
    memcpy(host + 256, fdh_be, 256);
    memcpy(host + 512, d_be, 256);
    if (crt) {
        memcpy(host + 768, dp_be, 128);
        memcpy(host + 896, dq_be, 128);
    }
    RC(key->table.ensure(sec::kGTabWords * sizeof(uint32_t)));
    uint8_t *st = key->dk.as<uint8_t>(kKeyStage);
    sec::TagKey *tk = key->dk.as<sec::TagKey>();
    hipStream_t s = ctx->stream();
    CK(hipMemcpyAsync(st, host, sizeof(host), hipMemcpyHostToDevice, s));
    int e = sec_launch_tag_setup(st, st + 256, st + 512, crt ? st + 768 : nullptr, crt ? st + 896 : nullptr, tk,
                                 key->table.as<uint32_t>(), s);
    if (e)
        return hip_fail((hipError_t)e, "sec_tag_setup");
    const uint32_t flag = crt ? 1u : 0u;
    CK(hipMemcpyAsync(&tk->crt, &flag, sizeof(flag), hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    key->has_tag = true;
    return SEC_OK;
}

int sec_bn_reduce_batch(sec_ctx *ctx, const sec_bn_key *key, const sec_msg *msgs, int64_t nmsgs, uint8_t *out,
                        unsigned flags)
{
    if (!ctx || !key || key->device != ctx->device)
        return SEC_EINVAL;
    const bool host = flags & SEC_F_HOST;
    const sec::BnKey *dk = key->dk.as<sec::BnKey>();
    bool prepared = false;
    return msg_batch(ctx, ctx->bn_plan, msgs, nmsgs, out, 256, flags,
                     (size_t)ctx->opt[O_SLAB_BYTES_DIGEST], 3, "sec_bn_reduce", kSegBytes,
                     [&](const uint8_t *base0, const Plan &plan, const SubPlan &sp, size_t idx, uint8_t *o,
                         hipStream_t s) {
                         if (!prepared) {
                             RC(bn_prepare(ctx, key, plan, host));
                             prepared = true;
                         }
                         return sec_launch_bn_reduce(dk, key->rpow.as<uint32_t>(), base0,
                                                     plan.meta.as<sec::MsgDesc>(sp.off_msgs), sp.nmsgs,
                                                     plan.meta.as<sec::SegDesc>(sp.off_segs), sp.nsegs,
                                                     plan.meta.as<sec::SegInfo>(sp.off_seginfo),
                                                     bn_part(ctx, idx, host), o, s);
                     });
}

int sec_apdp_tag_batch(sec_ctx *ctx, const sec_bn_key *key, const sec_msg *msgs, int64_t nmsgs, uint8_t *tags,
                       unsigned flags)
{
    if (!ctx || !key || key->device != ctx->device)
        return SEC_EINVAL;
    if (!key->has_tag)
        return SEC_ENOTAG;
    const bool host = flags & SEC_F_HOST;
    const sec::TagKey *tk = key->dk.as<sec::TagKey>();
    const uint32_t *table = key->table.as<uint32_t>();
    bool prepared = false;
    return msg_batch(ctx, ctx->bn_plan, msgs, nmsgs, tags, 256, flags,
                     (size_t)ctx->opt[O_SLAB_BYTES_DIGEST], 3, "sec_apdp_tag", kSegBytes,
                     [&](const uint8_t *base0, const Plan &plan, const SubPlan &sp, size_t idx, uint8_t *o,
                         hipStream_t s) {
                         if (!prepared) {
                             RC(bn_prepare(ctx, key, plan, host));
                             prepared = true;
                         }
                         return sec_launch_apdp_tag(tk, table, key->rpow.as<uint32_t>(), base0,
                                                    plan.meta.as<sec::MsgDesc>(sp.off_msgs), sp.nmsgs,
                                                    plan.meta.as<sec::SegDesc>(sp.off_segs), sp.nsegs,
                                                    plan.meta.as<sec::SegInfo>(sp.off_seginfo),
                                                    bn_part(ctx, idx, host), o, s);
                     });
}

int sec_bn_modexp_batch(sec_ctx *ctx, const sec_bn_key *key, const uint8_t *bases, const uint8_t *exps,
                        uint32_t exp_bytes, int64_t count, uint8_t *out, unsigned flags)
{
    if (!ctx || !key || key->device != ctx->device || count < 0 || count >= (int64_t)INT32_MAX ||
        (count > 0 && (!bases || !exps || !out)) || exp_bytes < 1 || exp_bytes > 4096 ||
        (flags & ~(SEC_F_HOST | SEC_F_ASYNC)))
        return SEC_EINVAL;
    if (count == 0)
        return SEC_OK;
    const sec::BnKey *dk = key->dk.as<sec::BnKey>();
    return dense_batch(ctx, {{bases, (size_t)count * 256}, {exps, (size_t)count * exp_bytes}}, out,
                       (size_t)count * 256, flags, "sec_bn_modexp_kernel",
                       [&](const std::vector<const uint8_t *> &in, uint8_t *o, hipStream_t s) {
                           return sec_launch_bn_modexp(dk, in[0], in[1], exp_bytes, (uint32_t)count, o, s);
                       });
}

int sec_bn_crt_modexp_batch(sec_ctx *ctx, const sec_bn_key *key, const uint8_t *bases, const uint8_t *exps_p,
                            const uint8_t *exps_q, uint32_t exp_bytes, int64_t count, uint8_t *out, unsigned flags)
{
    if (!ctx || !key || key->device != ctx->device || count < 0 || count >= (int64_t)INT32_MAX ||
        (count > 0 && (!bases || !exps_p || !exps_q || !out)) || exp_bytes < 1 || exp_bytes > 4096 ||
        (flags & ~(SEC_F_HOST | SEC_F_ASYNC)))
        return SEC_EINVAL;
    if (!key->has_crt)
        return SEC_ENOCRT;
    if (count == 0)
        return SEC_OK;
    const sec::TagKey *tk = key->dk.as<sec::TagKey>();
    const size_t eb = (size_t)count * exp_bytes;
    return dense_batch(ctx, {{bases, (size_t)count * 256}, {exps_p, eb}, {exps_q, eb}}, out, (size_t)count * 256,
                       flags, "sec_bn_crt_modexp_kernel",
                       [&](const std::vector<const uint8_t *> &in, uint8_t *o, hipStream_t s) {
                           return sec_launch_bn_crt_modexp(tk, in[0], in[1], in[2], exp_bytes, (uint32_t)count, o, s);
                       });
}

int sec_apdp_gpow_batch(sec_ctx *ctx, const sec_bn_key *key, const uint8_t *exps, uint32_t exp_bytes, int64_t count,
                        uint8_t *out, unsigned flags)
{
    if (!ctx || !key || key->device != ctx->device || count < 0 || count >= (int64_t)INT32_MAX ||
        (count > 0 && (!exps || !out)) || exp_bytes < 1 || exp_bytes > 256 || (flags & ~(SEC_F_HOST | SEC_F_ASYNC)))
        return SEC_EINVAL;
    if (!key->has_tag)
        return SEC_ENOTAG;
    if (count == 0)
        return SEC_OK;
    const sec::TagKey *tk = key->dk.as<sec::TagKey>();
    const uint32_t *table = key->table.as<uint32_t>();
    return dense_batch(ctx, {{exps, (size_t)count * exp_bytes}}, out, (size_t)count * 256, flags,
                       "sec_apdp_gpow_kernel", [&](const std::vector<const uint8_t *> &in, uint8_t *o, hipStream_t s) {
                           return sec_launch_apdp_gpow(tk, table, in[0], exp_bytes, (uint32_t)count, o, s);
                       });
}

int sec_bn_mulmod_batch(sec_ctx *ctx, const sec_bn_key *key, const uint8_t *a, const uint8_t *b, int64_t count,
                        uint8_t *out, unsigned flags)
{
    if (!ctx || !key || key->device != ctx->device || count < 0 || count >= (int64_t)INT32_MAX ||
        (count > 0 && (!a || !b || !out)) || (flags & ~(SEC_F_HOST | SEC_F_ASYNC)))
        return SEC_EINVAL;
    if (count == 0)
        return SEC_OK;
    const sec::BnKey *dk = key->dk.as<sec::BnKey>();
    return dense_batch(ctx, {{a, (size_t)count * 256}, {b, (size_t)count * 256}}, out, (size_t)count * 256, flags,
                       "sec_bn_mulmod_kernel",
                       [&](const std::vector<const uint8_t *> &in, uint8_t *o, hipStream_t s) {
                           return sec_launch_bn_mulmod(dk, in[0], in[1], (uint32_t)count, o, s);
                       });
}

// ---------------------------------------------------------------------------
int sec_decode_batch(sec_ctx *ctx, const sec_dec_chunk *chunks, int64_t nchunks, const int32_t *sharenums,
                     const uint64_t *block_offs, const uint8_t *blocks, uint8_t *out, unsigned flags)
{
    return sec_decode_batch_ex(ctx, chunks, nchunks, sharenums, block_offs, nullptr, blocks, out, flags);
}

namespace {
constexpr uint64_t kJoinPiece = (uint64_t)1 << 20;  // host-join copies per task
int decode_core(sec_ctx *ctx, const sec_dec_chunk *chunks, int64_t nchunks, const int32_t *sharenums,
                const uint64_t *block_offs, const uint64_t *block_avail, const uint8_t *blocks, uint8_t *out,
                unsigned flags, bool rows_only);
}  // namespace

int sec_decode_batch_ex(sec_ctx *ctx, const sec_dec_chunk *chunks, int64_t nchunks, const int32_t *sharenums,
                        const uint64_t *block_offs, const uint64_t *block_avail, const uint8_t *blocks, uint8_t *out,
                        unsigned flags)
{
    return decode_core(ctx, chunks, nchunks, sharenums, block_offs, block_avail, blocks, out, flags, false);
}

namespace {
bool primary_lost(const sec_dec_chunk &c, const int32_t *sharenums)
{
    for (int j = 0; j < c.k; ++j)
        if (sharenums[c.slot0 + j] >= c.k)
            return true;
    return false;
}

// The present primaries of chunk c, from the caller's blocks to their rows in `out` (rows
// clipped to the chunk's n bytes, zero past a slot's avail), as 1 MiB tasks on the pool.
void submit_row_copies(sec::TaskPool &tp, sec::TaskPool::Group &g, const sec_dec_chunk &c, const int32_t *sharenums,
                       const uint64_t *block_offs, const uint64_t *block_avail, const uint8_t *blocks, uint8_t *out)
{
    const uint64_t n = (uint64_t)c.k * c.B - c.padlen;
    for (int q = 0; q < c.k; ++q) {
        const int j = sharenums[c.slot0 + q];
        if (j >= c.k || (uint64_t)j * c.B >= n)
            continue;
        const uint64_t row = std::min<uint64_t>(c.B, n - (uint64_t)j * c.B);
        const uint64_t av = std::min<uint64_t>(row, slot_avail(c, block_avail, q));
        uint8_t *dst = (uint8_t *)((uintptr_t)out + c.out_off + (uint64_t)j * c.B);
        const uint8_t *src = (const uint8_t *)((uintptr_t)blocks + block_offs[c.slot0 + q]);
        for (uint64_t o = 0; o < row; o += kJoinPiece) {
            const uint64_t len = std::min<uint64_t>(kJoinPiece, row - o);
            const uint64_t cp = o < av ? std::min<uint64_t>(len, av - o) : 0;
            tp.submit(g, [=] {
                if (cp)
                    memcpy(dst + o, src + o, cp);
                if (cp < len)
                    memset(dst + o + cp, 0, len - cp);
                return true;
            });
        }
    }
}

// A staged reassembly of host buffers (decode_core found them neither pinned nor lockable: e.g.
// one piece object per block), every chunk with a lost primary.  The present primaries go from
// the caller's blocks into `out` on the context's task threads, and a rows-only call computes
// the lost ones, reading the present primaries either
//  - back from `out`, once the copies are done, when those ranges would be page-locked (one
//    contiguous range per chunk in place of scattered pieces, read over PCIe in place), or
//  - from the caller's blocks, staged, while the copies run.
// Slots keep their indices; re-pointed offsets are absolute.
int join_staged(sec_ctx *ctx, const sec_dec_chunk *chunks, int64_t nchunks, const int32_t *sharenums,
                const uint64_t *block_offs, const uint64_t *block_avail, const uint8_t *blocks, uint8_t *out,
                unsigned flags)
{
    sec::TaskPool &tp = join_tasks(ctx);
    sec::TaskPool::Group g;
    std::vector<sec_dec_chunk> sub(chunks, chunks + nchunks);
    for (const sec_dec_chunk &c : sub)
        submit_row_copies(tp, g, c, sharenums, block_offs, block_avail, blocks, out);
    --ctx->staged_calls;  // the rows-only call counts this call's host path
    uint64_t nsl = 0;
    for (const sec_dec_chunk &c : sub)
        nsl = std::max<uint64_t>(nsl, c.slot0 + (uint64_t)c.k);
    std::vector<uint64_t> offs2(nsl, 0), avail2(nsl, 0);
    for (const sec_dec_chunk &c : sub) {
        const uint64_t n = (uint64_t)c.k * c.B - c.padlen;  // (padlen <= k*B: checked)
        for (int q = 0; q < c.k; ++q) {
            const uint64_t s = c.slot0 + (uint64_t)q;
            const int j = sharenums[s];
            // only a row `out` holds whole: a row cut by padlen keeps its own block, whose bytes
            // past the cut are not necessarily zero (any padlen <= k*B is legal)
            if (j < c.k && (uint64_t)(j + 1) * c.B <= n) {
                offs2[s] = (uintptr_t)out + c.out_off + (uint64_t)j * c.B;
                avail2[s] = c.B;
            } else {
                offs2[s] = (uintptr_t)blocks + block_offs[s];
                avail2[s] = slot_avail(c, block_avail, q);
            }
        }
    }
    // (a dry run: whether the rows-only call would page-lock these ranges; it locks them itself,
    // after the copies have landed)
    HostLock probe(ctx->stream());
    const bool from_out =
        probe.acquire(decode_ranges(sub.data(), (int64_t)sub.size(), sharenums, offs2.data(), avail2.data(), nullptr,
                                    out, false),
                      ctx->opt[O_REGISTER_MIN], !(flags & SEC_F_STAGED), true) != 0;
    int rc;
    if (from_out) {
        tp.wait(g);  // the present primaries are in `out` now
        rc = decode_core(ctx, sub.data(), (int64_t)sub.size(), sharenums, offs2.data(), avail2.data(), nullptr, out,
                         flags, true);
    } else {
        rc = decode_core(ctx, sub.data(), (int64_t)sub.size(), sharenums, block_offs, block_avail, blocks, out, flags,
                         true);
        tp.wait(g);
    }
    return rc;
}

// rows_only (a host reassembly whose present primaries the caller copies itself, see below):
// run the kernels for the recovered rows only, written to their output rows.
int decode_core(sec_ctx *ctx, const sec_dec_chunk *chunks, int64_t nchunks, const int32_t *sharenums,
                const uint64_t *block_offs, const uint64_t *block_avail, const uint8_t *blocks, uint8_t *out,
                unsigned flags, bool rows_only)
{
    if (!ctx || nchunks < 0 || (nchunks > 0 && (!chunks || !sharenums || !block_offs)) ||
        (flags & ~(SEC_F_HOST | SEC_F_ASYNC | SEC_F_RECOVER | SEC_F_STAGED)) ||
        ((flags & SEC_F_STAGED) && !(flags & SEC_F_HOST)))
        return SEC_EINVAL;
    if (nchunks == 0)
        return SEC_OK;
    if (nchunks >= (int64_t)UINT32_MAX)
        return SEC_EINVAL;
    bool host = flags & SEC_F_HOST;
    const bool recover = flags & SEC_F_RECOVER;
    RC(set_dev(ctx));

    // _fec.Decoder.decode / easyfec.Decoder.decode preconditions
    uint64_t total_slots = 0, total_out = 0;
    for (int64_t i = 0; i < nchunks; ++i) {
        const sec_dec_chunk &c = chunks[i];
        if (c.k < 1 || c.m < c.k || c.m > 256)
            return SEC_EKM;
        if (c.B >= (1ull << 31))
            return SEC_ESIZE;
        if (c.padlen > (uint64_t)c.k * c.B)
            return SEC_EPADLEN;
        RC(check_sharenums(c.k, c.m, sharenums + c.slot0));
        total_slots = std::max<uint64_t>(total_slots, c.slot0 + (uint64_t)c.k);
        total_out += dec_nout(c, sharenums, recover);
    }
    if (total_out == 0)
        return SEC_OK;
    // (blocks and out may be NULL: block_offs / out_off are then absolute addresses)
    // A reassembly of host buffers leaves the present primaries to the host (the context's task
    // threads copy them from the caller's blocks into `out`) and moves only what the GPU computes
    // over PCIe: the recovered rows, e * B per chunk instead of the whole chunk (option
    // SEC_HOST_JOIN = 0: the GPU writes every output byte).  Chunks with every primary present
    // never reach the GPU.  Buffers the device can use in place (pinned, or pageable and
    // locked for the call) keep the concurrent form below instead: the kernels write the
    // recovered rows in place while the copy threads join the present rows.
    const bool join = host && !recover && ctx->opt[O_HOST_JOIN] != 0;
    if (join && !rows_only) {
        // chunks with every primary present: copies on the task threads only (no GPU, and their
        // buffers are not page-locked), the rest of the call running meanwhile
        std::vector<sec_dec_chunk> sub;
        for (int64_t i = 0; i < nchunks; ++i)
            if (primary_lost(chunks[i], sharenums))
                sub.push_back(chunks[i]);
        if ((int64_t)sub.size() < nchunks) {
            sec::TaskPool &tp = join_tasks(ctx);
            sec::TaskPool::Group g;
            for (int64_t i = 0; i < nchunks; ++i)
                if (!primary_lost(chunks[i], sharenums))
                    submit_row_copies(tp, g, chunks[i], sharenums, block_offs, block_avail, blocks, out);
            const int rc = sub.empty() ? SEC_OK
                                       : decode_core(ctx, sub.data(), (int64_t)sub.size(), sharenums, block_offs,
                                                     block_avail, blocks, out, flags, false);
            tp.wait(g);
            return rc;
        }
    }
    // pinned (or lockable) caller buffers: the device path on them directly (see encode_impl)
    HostLock lock(ctx->stream());
    bool direct = false;
    if (host &&
        host_direct(ctx, decode_ranges(chunks, nchunks, sharenums, block_offs, block_avail, blocks, out, recover),
                    lock, flags)) {
        host = false;
        direct = true;
        flags &= ~(SEC_F_HOST | SEC_F_ASYNC);
    }
    if (join && !rows_only && !direct)
        return join_staged(ctx, chunks, nchunks, sharenums, block_offs, block_avail, blocks, out, flags);
    // the primaries a joining call copies on the host: row j of chunk i from the slot holding
    // primary j, up to that slot's avail (zero past it), rows clipped to the chunk's n bytes
    std::vector<sec::CopyJob> joins;
    if (join && !rows_only) {
        for (int64_t i = 0; i < nchunks; ++i) {
            const sec_dec_chunk &c = chunks[i];
            const uint64_t n = (uint64_t)c.k * c.B - c.padlen;
            for (int q = 0; q < c.k; ++q) {
                const int j = sharenums[c.slot0 + q];
                if (j >= c.k || (uint64_t)j * c.B >= n)
                    continue;
                const uint64_t row = std::min<uint64_t>(c.B, n - (uint64_t)j * c.B);
                const uint64_t av = std::min<uint64_t>(row, slot_avail(c, block_avail, q));
                uint8_t *dst = out + c.out_off + (uint64_t)j * c.B;
                joins.push_back(sec::CopyJob{dst, blocks + block_offs[c.slot0 + q], av});
                if (av < row)
                    joins.push_back(sec::CopyJob{dst + av, nullptr, row - av});
            }
        }
    }
    // staged joining calls run the kernels in recover mode (dense rows); direct ones write the
    // recovered rows in place with the copies switched off (nocopy)
    const bool prec = recover || (join && host);
    const bool nocopy = join && direct;

    // Plan key (see sec_encode_batch): host mode keys on shapes + sharenums only (its slots
    // are staged densely, zero-filled past their avail); device mode on every descriptor,
    // sharenum, block offset and avail.
    Plan &plan = ctx->dec_plan;
    std::vector<uint8_t> key;
    if (host) {
        for (int64_t i = 0; i < nchunks; ++i) {
            const sec_dec_chunk &c = chunks[i];
            const size_t o = key.size();
            key.resize(o + 24 + (size_t)c.k * 4);
            memcpy(key.data() + o, &c.B, 8);
            memcpy(key.data() + o + 8, &c.padlen, 8);
            memcpy(key.data() + o + 16, &c.k, 4);
            memcpy(key.data() + o + 20, &c.m, 4);
            memcpy(key.data() + o + 24, sharenums + c.slot0, (size_t)c.k * 4);
        }
    } else {
        const size_t kc = sizeof(sec_dec_chunk) * (size_t)nchunks;
        const size_t ka = block_avail ? total_slots * 8 : 0;
        key.resize(kc + total_slots * (4 + 8) + ka);
        memcpy(key.data(), chunks, kc);
        memcpy(key.data() + kc, sharenums, total_slots * 4);
        memcpy(key.data() + kc + total_slots * 4, block_offs, total_slots * 8);
        if (ka)
            memcpy(key.data() + kc + total_slots * 12, block_avail, ka);
    }
    // ASYNC does not change the plan; whether an avail array came does (0x10000), and how a
    // joining call runs the kernels (recover 0x4 / nocopy 0x20000)
    const unsigned kflags = (flags & ~(SEC_F_ASYNC | SEC_F_STAGED)) | (!host && block_avail ? 0x10000u : 0u) |
                            (prec ? SEC_F_RECOVER : 0u) | (nocopy ? 0x20000u : 0u);
    key.insert(key.end(), (const uint8_t *)&kflags, (const uint8_t *)&kflags + sizeof(unsigned));
    const bool reuse = plan.valid && plan.gen == ctx->dec_tabs.gen && plan.key == key;
    DecLayout L;
    if (!reuse || host)
        L = dec_layout(chunks, nchunks, sharenums);
    if (!reuse) {
        plan.valid = false;
        RC(build_decode_plan(ctx, chunks, nchunks, block_offs, block_avail, L, host, prec, nocopy));
        plan.key.swap(key);
        plan.valid = true;
    }
    ctx->syn_chunks += plan.nsyn;
    ctx->direct_chunks += plan.ndirect;
    ctx->fused_chunks += plan.nfused;

    if (!host) {
        hipEvent_t t0 = nullptr;
        RC(ctx->syn.ensure(plan.subs[0].syn_bytes));
        RC(timing_begin(ctx, &t0, ctx->stream()));
        RC(launch_decode_sub(ctx, plan, plan.subs[0], blocks, out, ctx->stream(), ctx->syn.as<uint8_t>()));
        RC(timing_end(ctx, t0, 1, ctx->stream()));
        if (nocopy)  // the present primaries, host to host, while the kernels run
            pool(ctx).run_copies(joins);
        if (!(flags & SEC_F_ASYNC))
            CK(hipStreamSynchronize(ctx->stream()));
        return SEC_OK;
    }
    auto gather = [&](const SubPlan &sp, char *stage, std::vector<sec::CopyJob> &jobs) {
        uint64_t o = 0;
        for (int64_t i = sp.c0; i < sp.c1; ++i) {
            const sec_dec_chunk &c = chunks[i];
            for (int s = 0; s < c.k; ++s) {
                const int from = L.perm[L.first[i] + s];
                const uint64_t av = slot_avail(c, block_avail, from);
                jobs.push_back(sec::CopyJob{stage + o, blocks + block_offs[c.slot0 + from], av});
                if (av < c.B)  // the slot's bytes past its avail are zero
                    jobs.push_back(sec::CopyJob{stage + o + av, nullptr, c.B - av});
                o += c.B;
            }
        }
    };
    auto scatter = [&](const SubPlan &sp, char *stage, std::vector<sec::CopyJob> &jobs) {
        uint64_t o = 0;
        for (int64_t i = sp.c0; i < sp.c1; ++i) {
            const sec_dec_chunk &c = chunks[i];
            const uint64_t nout = dec_nout(c, sharenums, prec);
            if (!join) {
                jobs.push_back(sec::CopyJob{out + c.out_off, stage + o, nout});
            } else {  // the recovered rows (dense, in primary order) to their output rows
                const uint64_t n = (uint64_t)c.k * c.B - c.padlen;
                uint64_t r = 0;
                for (int s = 0; s < c.k; ++s) {  // slot s of the normalised layout = primary s
                    if (L.idx[L.first[i] + s] < c.k)
                        continue;
                    if ((uint64_t)s * c.B < n)
                        jobs.push_back(sec::CopyJob{out + c.out_off + (uint64_t)s * c.B, stage + o + r * c.B,
                                                    std::min<uint64_t>(c.B, n - (uint64_t)s * c.B)});
                    ++r;
                }
            }
            o += nout;
        }
    };
    auto launch = [&](const SubPlan &sp, uint8_t *din, uint8_t *dout, hipStream_t s) {
        uint8_t *syn = nullptr;
        if (sp.syn_bytes)
            for (Slot &slot : ctx->slots)  // the unit's slot: its own syndrome scratch
                if (slot.s == s) {
                    RC(slot.dsyn.ensure(sp.syn_bytes));
                    syn = slot.dsyn.as<uint8_t>();
                }
        return launch_decode_sub(ctx, plan, sp, din, dout, s, syn);
    };
    RC(run_pipeline(ctx, plan, gather, scatter, launch, true));
    if (join)  // the present primaries, host to host
        pool(ctx).run_copies(joins);
    return SEC_OK;
}
}  // namespace

// ---------------------------------------------------------------------------
int sec_malloc(sec_ctx *ctx, size_t bytes, void **dptr)
{
    if (!ctx || !dptr)
        return SEC_EINVAL;
    RC(set_dev(ctx));
    if (hipMalloc(dptr, bytes ? bytes : 1) != hipSuccess)
        return SEC_ENOMEM;
    return SEC_OK;
}

int sec_free(sec_ctx *ctx, void *dptr)
{
    if (!ctx)
        return SEC_EINVAL;
    RC(set_dev(ctx));
    CK(hipFree(dptr));
    return SEC_OK;
}

int sec_host_alloc(sec_ctx *ctx, size_t bytes, void **hptr)
{
    if (!ctx || !hptr)
        return SEC_EINVAL;
    RC(set_dev(ctx));
    if (hipHostMalloc(hptr, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess)
        return SEC_ENOMEM;
    return SEC_OK;
}

int sec_host_free(sec_ctx *ctx, void *hptr)  // ctx unused: may be NULL (or already destroyed)
{
    (void)ctx;
    CK(hipHostFree(hptr));
    return SEC_OK;
}

int sec_host_register(sec_ctx *ctx, void *hptr, size_t bytes)
{
    if (!ctx || !hptr || !bytes)
        return SEC_EINVAL;
    RC(set_dev(ctx));
    CK(hipHostRegister(hptr, bytes, hipHostRegisterDefault));
    return SEC_OK;
}

int sec_host_unregister(sec_ctx *ctx, void *hptr)  // ctx unused: may be NULL
{
    (void)ctx;
    if (!hptr)
        return SEC_EINVAL;
    CK(hipHostUnregister(hptr));
    return SEC_OK;
}

int sec_ctx_decode_paths(sec_ctx *ctx, int64_t *syndrome, int64_t *direct)
{
    if (!ctx)
        return SEC_EINVAL;
    if (syndrome)
        *syndrome = ctx->syn_chunks;
    if (direct)
        *direct = ctx->direct_chunks;
    return SEC_OK;
}

int sec_ctx_decode_methods(sec_ctx *ctx, int64_t *fused, int64_t *pair, int64_t *two_kernel, int64_t *direct)
{
    if (!ctx)
        return SEC_EINVAL;
    if (fused)
        *fused = ctx->fused_chunks;
    if (pair)  // the one-kernel wave pair is archived (round 5): always 0
        *pair = 0;
    if (two_kernel)
        *two_kernel = ctx->syn_chunks - ctx->fused_chunks;
    if (direct)
        *direct = ctx->direct_chunks;
    return SEC_OK;
}

int sec_host_pinned_bytes(int64_t *loaned, int64_t *idle)
{
    PinPool::get().stats(loaned, idle);
    return SEC_OK;
}

int sec_ctx_host_paths(sec_ctx *ctx, int64_t *zero_copy, int64_t *registered, int64_t *staged)
{
    if (!ctx || !zero_copy || !registered || !staged)
        return SEC_EINVAL;
    *zero_copy = ctx->zero_copy_calls;
    *registered = ctx->registered_calls;
    *staged = ctx->staged_calls;
    return SEC_OK;
}

int sec_memcpy(sec_ctx *ctx, void *dst, const void *src, size_t bytes, int kind)
{
    if (!ctx || (bytes && (!dst || !src)) || kind < 0 || kind > 2)
        return SEC_EINVAL;
    RC(set_dev(ctx));
    static const hipMemcpyKind kinds[3] = {hipMemcpyHostToDevice, hipMemcpyDeviceToHost, hipMemcpyDeviceToDevice};
    if (bytes) {
        CK(hipMemcpyAsync(dst, src, bytes, kinds[kind], ctx->stream()));
        CK(hipStreamSynchronize(ctx->stream()));
    }
    return SEC_OK;
}

// Host-to-host copies on the context's copy threads (the calling thread takes part): the join of
// a reassembled chunk's rows into one output buffer -- present primaries straight from the
// caller's piece objects, recovered rows from a result buffer -- without the caller's
// single-threaded join (easyfec's b"".join, /root/reference/storb/util/piece.py:196-197).
// src == 0: zero-fill.
int sec_host_copy(sec_ctx *ctx, const sec_copy *jobs, int64_t njobs)
{
    if (!ctx || njobs < 0 || (njobs > 0 && !jobs))
        return SEC_EINVAL;
    std::vector<sec::CopyJob> cj;
    cj.reserve((size_t)njobs);
    for (int64_t i = 0; i < njobs; ++i) {
        if (!jobs[i].len)
            continue;
        if (!jobs[i].dst)
            return SEC_EINVAL;
        cj.push_back(sec::CopyJob{(void *)(uintptr_t)jobs[i].dst, (const void *)(uintptr_t)jobs[i].src,
                                  (size_t)jobs[i].len});
    }
    join_tasks(ctx).run_copies(cj);
    return SEC_OK;
}

int sec_memset(sec_ctx *ctx, void *dptr, int value, size_t bytes)
{
    if (!ctx || (bytes && !dptr))
        return SEC_EINVAL;
    RC(set_dev(ctx));
    if (bytes) {
        CK(hipMemsetAsync(dptr, value, bytes, ctx->stream()));
        CK(hipStreamSynchronize(ctx->stream()));
    }
    return SEC_OK;
}

}  // extern "C"
