// kernels.hpp — device-side descriptors shared by kernels.hip and api.cpp.
//
// Work decomposition.  A "tile" is one workgroup of L lanes over a run of
// L*16*U consecutive byte positions t of ONE chunk's blocks (U = 1: the kernels keep U as a
// template parameter, but only U = 1 is built; L any multiple of 64 up to 1024),
// and a group of up to 8 output rows (parity rows for encode, missing data rows
// for decode).  Each lane owns 16 consecutive positions per u-step, so every
// wave reads one coalesced 1 KiB run from each of the k input blocks and
// writes one 1 KiB run per output row.  Tiles cover [0, valid) of a chunk
// (valid = length of its last, possibly short, data block); the < padlen
// positions in [valid, B) are computed byte by byte by the chunk's last tile
// (Tile::ntail).  Chunks too small for a tile (valid < 16) become "tail items",
// one thread per position, in a separate launch.
#pragma once
#include <stdint.h>

namespace sec {

constexpr int kLanes = 256;         // threads per workgroup
constexpr int kLaneBytes = 16;      // bytes per lane per u-step (dwordx4)
constexpr int kStepBytes = kLanes * kLaneBytes;  // 4 KiB per u-step
constexpr int kMaxRows = 8;         // output rows per tile (accumulator groups)
constexpr int kTabDwords = 5;       // v_perm tables per GF coefficient
constexpr int kBatchVecs = 16;      // 16 B vectors a lane loads per batch (SEC_ENC/DEC_BATCH):
                                    // a tile has U > 1 only if k * U <= kBatchVecs
// Largest workgroup of a tile kernel with `rows` output rows (its launch bound, which also
// caps its VGPRs: 1024 lanes leave 128 per lane).  Groups of more than 4 rows are bound by
// SEC_LB_WIDE_ROWS lanes (A/B knob); the plan clamps its tile widths to this.
#ifndef SEC_LB_WIDE_ROWS
#define SEC_LB_WIDE_ROWS 1024
#endif
constexpr int max_lanes(int rows, int U) { return U != 1 ? kLanes : (rows > 4 ? SEC_LB_WIDE_ROWS : 1024); }

// One encode chunk, device copy (48 B).
struct EncDesc {
    uint64_t in_off;      // chunk start in `in`
    uint64_t par_off;     // first parity block in `parity`
    uint64_t par_stride;  // bytes between parity blocks
    uint32_t B;           // block bytes = ceil(n/k)
    uint32_t k;           // data blocks
    uint32_t p;           // parity blocks (m - k)
    uint32_t tab;         // dword offset of this chunk's tables, layout [j][r][5]
    uint32_t valid;       // n - (k-1)*B: bytes of the last (zero-padded) data block
    uint32_t pad;
};

// One decode chunk, device copy (40 B).
struct DecDesc {
    uint64_t out_off;  // reassembled chunk start in `out`
    uint64_t n;        // bytes to write = k*B - padlen
    uint32_t B;
    uint32_t k;
    uint32_t e;        // missing primaries (rows recovered)
    uint32_t tab;      // dword offset of tables, layout [slot][missing][5]
    uint32_t slot0;    // first entry in slot_off / slot_row / miss_row
    uint32_t valid;    // positions [0, valid) where every output row is writable and every slot
                       // readable: min(last output row's length, every slot's avail), clamped to [0, B)
};

// Per-slot metadata of a decode launch (device arrays).  Slot c of a chunk is entry
// slot0 + c; a chunk's recovered rows are miss[slot0 .. slot0 + e).
struct DecSlots {
    const uint64_t *off;    // block address: blocks + off[slot]
    const uint32_t *row;    // output row a present primary is copied to, or 0xFFFFFFFF
    const uint32_t *miss;   // output row of each recovered (missing) primary
    const uint32_t *avail;  // bytes of the block that exist in memory; the rest read as zero
};

// One chunk of a syndrome decode (kernels_bs.hip sec_syndrome_bs_kernel, sec_decode_bs_kernel; 56 B).  Block j of
// the chunk (data j < k, parity row r at j = k + r) is at blocks + off[slot0 + j] with
// avail[slot0 + j] readable bytes, when its bit in dmask / pmask is set.
struct SynDesc {
    uint64_t out_off;  // reassembled chunk in `out`: present primaries are copied there (tile flag)
    uint64_t syn_off;  // syndrome q (of the q-th present parity row) at syn + syn_off + q * syn_stride(B)
    uint64_t dmask;    // bit j: data block j present (k <= 64)
    uint64_t pmask;    // bit r: parity row r present (m - k <= 64)
    uint32_t B;
    uint32_t last;     // bytes of output row k-1 (n - (k-1)*B): its stores stop there (recover-only: B)
    uint32_t slot0;
    uint32_t wq0;      // masks[wq0 + q]: the scaling w of syndrome q (scale_mask)
    uint32_t zq0;      // fused kernel: masks[zq0 + t], the scaling z of the t-th lost row
    uint32_t flags;    // fused kernel: bit 1 = recover-only (recovered rows by rank)
};

struct SynSlots {
    const uint64_t *off;
    const uint32_t *avail;
    const uint64_t *masks;  // scalings of both phases (scale_mask layout)
};

// One chunk of a syndrome decode, phase 2 (kernels_bs.hip sec_solve_bs_kernel; 48 B): the lost
// data rows from the scaled bit-sliced syndromes.
struct SolveDesc {
    uint64_t out_off;
    uint64_t syn_off;  // as SynDesc
    uint64_t lost;     // bit l: data row l is recovered
    uint64_t pmask;    // bit r: parity row r present (syndrome q = the q-th set bit)
    uint32_t B;
    uint32_t last;     // bytes output row k-1 holds (reassembly; recover-only: B)
    uint32_t zq0;      // masks[zq0 + t]: the scaling z of the t-th recovered row (ascending)
    uint32_t recover;  // 1: recovered row t at out_off + t * B (else row l at out_off + l * B)
};

// Syndromes are stored bit-sliced (a lane's 8 planes where its 32 bytes would be), at the
// lanes' unclamped positions: rows of whole 2048-position wave spans.
constexpr uint64_t kSynSpan = 2048;
constexpr uint64_t syn_stride(uint64_t B) { return (B + kSynSpan - 1) / kSynSpan * kSynSpan; }

struct Tile {
    uint32_t chunk;  // descriptor index
    uint32_t t0;     // first byte position within the block
    uint32_t r0;     // first output row of this tile's row group
    uint32_t ntail;  // on the chunk's last tile of the row group: B - valid, the ragged
                     // positions [valid, B) it also computes byte by byte; else 0
};

// One byte position handled by the tail kernels.
struct TailItem {
    uint32_t chunk;
    uint32_t t;
};

// One SHA-1 message (a piece): `len` bytes at bases[base] + off, of which the
// first `avail` exist in memory; the rest read as zero (zfec's padding of the
// last data block, which is part of that piece's bytes).
struct MsgDesc {
    uint64_t off;
    uint64_t len;
    uint64_t avail;
    uint32_t base;  // 0 or 1: which of the launch's two base pointers
    uint32_t pad;
};

}  // namespace sec

// launchers (kernels.hip); all enqueue on `stream` and return hipError_t as int
extern "C++" {
// Timing: the next launch's dispatch records `start`, every launch records `stop` (both
// hipEvent_t, or null), until the next call; returns the launches since the previous call.
int sec_launch_events(void *start, void *stop);
// For launchers in other translation units: the events the next dispatch records (as above),
// counted as a launch; pass them to hipExtLaunchKernelGGL.
void sec_next_launch_events(void **start, void **stop);
int sec_launch_expand(const uint8_t *coef, uint32_t ncoef, uint32_t *tabs, void *stream);
// wide: k > kBatchVecs / U (U must be 1): the kernels that load the blocks in several batches
int sec_launch_encode(int rows, int U, int wide, int lanes, const uint8_t *in, uint8_t *par,
                      const sec::EncDesc *descs, const sec::Tile *tiles, uint32_t ntiles, const uint32_t *tabs,
                      void *stream);
// Bit-sliced compile-time-matrix encode (kernels_bs.hip) for the shapes sec_bs_shape knows
// (else -1; rows = 0: the first kernel of that (k, m), else the one of `rows` rows per group):
// all of [0, B) of chunks with B >= 16: group 0 for the one-group shapes, tiles of `lanes`
// (64..256) lanes over lanes / 64 wave spans of sec_bs_span() positions; group -2 for zfec(64,96)
// (two row groups): both groups of one span per two-wave workgroup, one tile per span, `lanes`
// ignored
int sec_bs_shape(int k, int m, int rows = 0);
int sec_bs_groups(int shape);
int sec_bs_rows(int shape);
uint32_t sec_bs_span();
int sec_launch_encode_bs(int shape, int group, int lanes, const uint8_t *in, uint8_t *par, const sec::EncDesc *descs,
                         const sec::Tile *t, uint32_t ntiles, void *stream);
// Syndrome decode, phase 1, for the shapes sec_syn_shape knows (else -1): tiles as the bit-sliced
// encode's (r0 = the row group's first parity row; ntail bit 0 = this tile also copies the
// present primaries to `out`)
int sec_syn_shape(int k, int m);
int sec_launch_syndrome_bs(int shape, int lanes, const uint8_t *blocks, uint8_t *out, uint8_t *syn,
                           const sec::SynDesc *descs, const sec::Tile *t, uint32_t ntiles, sec::SynSlots sl,
                           void *stream);
// Phase 1 of zfec(64,96) chunks with present parity rows in both groups: one two-wave workgroup per
// span (tile t0; ntail bit 0 = copy the present primaries), wave g group g (sec_syn_pair shapes)
int sec_launch_syndrome_bs_pair(int shape, const uint8_t *blocks, uint8_t *out, uint8_t *syn, const sec::SynDesc *descs,
                                const sec::Tile *t, uint32_t ntiles, sec::SynSlots sl, void *stream);
// Both phases in one kernel (e <= 16 and every present parity row in the tile's row group r0):
// the syndromes stay in registers
int sec_launch_decode_bs(int shape, int lanes, const uint8_t *blocks, uint8_t *out, const sec::SynDesc *descs,
                         const sec::Tile *t, uint32_t ntiles, sec::SynSlots sl, void *stream);
// The shapes with the two-wave phase-1 kernel (zfec(64,96): both 16-row parity groups)
int sec_syn_pair(int shape);
// Phase 2: the lost data rows of row group r0 / sec_solve_rows(shape) of each tile's chunk
int sec_solve_rows(int shape);
// Phase 2, one workgroup per span (tile t0): the span's e <= slots syndrome rows staged in LDS once,
// each wave one row group; on the shapes sec_solve_lds accepts (slots: a multiple of 8, <= 32)
int sec_solve_lds(int shape);
int sec_launch_solve_bs_lds(int shape, int slots, const uint8_t *syn, uint8_t *out, const sec::SolveDesc *descs,
                            const sec::Tile *t, uint32_t ntiles, const uint64_t *masks, void *stream);
int sec_launch_solve_bs(int shape, int lanes, const uint8_t *syn, uint8_t *out, const sec::SolveDesc *descs,
                        const sec::Tile *t, uint32_t ntiles, const uint64_t *masks, void *stream);
int sec_launch_encode_tail(const uint8_t *in, uint8_t *par, const sec::EncDesc *descs, const sec::TailItem *items,
                           uint32_t nitems, const uint32_t *tabs, void *stream);
// kb (4): the kernel variant whose load batch is kb slots (every chunk of the group has
// k <= kb; U = 1, not wide); 0: the default batch
int sec_launch_decode(int rows, int U, int wide, int lanes, const uint8_t *blocks, uint8_t *out,
                      const sec::DecDesc *descs, const sec::Tile *tiles, uint32_t ntiles, const uint32_t *tabs,
                      sec::DecSlots slots, void *stream, int kb = 0);
// split: sec_sha1_split_kernel (two waves per 64 messages: schedule and rounds) instead of
// one lane per message
int sec_launch_sha1(const uint8_t *base0, const uint8_t *base1, const sec::MsgDesc *msgs, uint32_t nmsgs,
                    uint8_t *digests, void *stream, int split = 0);
int sec_launch_decode_tail(const uint8_t *blocks, uint8_t *out, const sec::DecDesc *descs,
                           const sec::TailItem *items, uint32_t nitems, const uint32_t *tabs, sec::DecSlots slots,
                           void *stream);
}
