// ARCHIVED (round 5): bit-sliced kernels whose round-4 A/B lost to the shipped path; moved out of
// storb_amd/csrc/kernels_bs.hip with their launchers (they depend on that file's helpers, so they
// do not build alone).  Results: tools/archive/README.md.

// ===== sec_encode_bs_lds_kernel (SEC_BS_LDS: -9 % on C4, profiles/r04_c4_lds_ab.jsonl)
// ---- small chunks staged whole through LDS (C4's 64 KiB chunks) --------------------------------
// A chunk of n <= 64 KiB is read as ONE contiguous run (aligned 16-byte pieces, 256 lanes x 16
// loads in flight) into an LDS image of the chunk, instead of k block streams at zfec's unaligned
// block starts (C4: 10 streams of 6554 B per chunk, each 128-byte line at a block boundary read
// twice).  Lanes then take their positions' bytes of every block from the image (realigned from
// 8-aligned ds_read_b64s: a block starts at j*B, any alignment) and run the bit-sliced rows as
// sec_encode_bs_kernel.  Lane l owns positions 16 l and 4096 + 16 l (each moved back to end at B
// when past it, as there), so one 256-lane workgroup covers a chunk with B <= 8192.  The image's
// bytes past n are zero: zfec's padding of block k-1.
constexpr u32 kLdsChunk = 65536;  // largest chunk of the LDS-staged kernels

struct ChunkImg {
    u32x4 v[kLdsChunk / 16 + 4];  // the chunk, then zeros (block k-1 read past n)
};

__device__ __forceinline__ u32 align_bytes(u32 hi, u32 lo, u32 sh)
{
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// 16 bytes of the image at byte offset o (any alignment): three 8-aligned ds_read_b64, realigned
__device__ __forceinline__ void lds_piece(const ChunkImg &img, u32 o, u32 *x)
{
    const uint2 *p = reinterpret_cast<const uint2 *>(img.v) + (o >> 3);
    const uint2 a = p[0], b = p[1], c = p[2];
    const u32 sh = o & 3;
    if (o & 4) {
        x[0] = align_bytes(b.x, a.y, sh);
        x[1] = align_bytes(b.y, b.x, sh);
        x[2] = align_bytes(c.x, b.y, sh);
        x[3] = align_bytes(c.y, c.x, sh);
    } else {
        x[0] = align_bytes(a.y, a.x, sh);
        x[1] = align_bytes(b.x, a.y, sh);
        x[2] = align_bytes(b.y, b.x, sh);
        x[3] = align_bytes(c.x, b.y, sh);
    }
}

template <int K, int M, int NR, int J>
__device__ __forceinline__ void lds_block(u32 (&acc)[NR * 8], const ChunkImg &img, u32 B, u32 ta, u32 tb)
{
    u32 x[8];
    lds_piece(img, (u32)J * B + ta, x);
    lds_piece(img, (u32)J * B + tb, x + 4);
    transpose8(x);
    u32 lo[16], hi[16];
    subsets(x[0], x[1], x[2], x[3], lo);
    subsets(x[4], x[5], x[6], x[7], hi);
    block_rows<K, M, 0, J, J == 0>(std::make_integer_sequence<int, NR * 8>{}, acc, lo, hi);
}

template <int K, int M, int NR, int... Js>
__device__ __forceinline__ void lds_blocks(std::integer_sequence<int, Js...>, u32 (&acc)[NR * 8], const ChunkImg &img,
                                           u32 B, u32 ta, u32 tb)
{
    (lds_block<K, M, NR, Js>(acc, img, B, ta, tb), ...);
}

// One workgroup (256 lanes) per chunk: every parity row (M - K <= 8).
template <int K, int M>
__global__ __launch_bounds__(256) void sec_encode_bs_lds_kernel(const u8 *__restrict__ in, u8 *__restrict__ par,
                                                                const sec::EncDesc *__restrict__ descs,
                                                                const sec::Tile *__restrict__ tiles)
{
    constexpr int NR = M - K;
    __shared__ ChunkImg img;
    const sec::EncDesc d = descs[tiles[blockIdx.x].chunk];
    const u32 B = d.B, n = (u32)(K - 1) * B + d.valid, nf = n / 16;  // nf >= 1 (B >= 16)
    const u8 *src = in + d.in_off;
    const u32 t = threadIdx.x;
    // every lane issues all its loads before any LDS store (pieces past the chunk repeat its last
    // whole piece, not stored): 16 x 1 KiB coalesced runs per wave in flight
    u32x4 r[kLdsChunk / 16 / 256];
#pragma unroll
    for (int i = 0; i < (int)(kLdsChunk / 16 / 256); ++i)
        r[i] = ld16<true>(src + 16 * min(t + 256u * i, nf - 1));
#pragma unroll
    for (int i = 0; i < (int)(kLdsChunk / 16 / 256); ++i)
        if (t + 256u * i < nf)
            img.v[t + 256u * i] = r[i];
    if (t < 4)  // the partial last piece (zero past n), then zeros
        img.v[nf + t] = t == 0 && n % 16 ? ld16_avail<true>(src, 16 * nf, n) : u32x4{0, 0, 0, 0};
    __syncthreads();
    const u32 ta = min(16 * t, B - 16), tb = min(16 * t + 4096, B - 16);
    if (16 * t >= B)  // both pieces would repeat a neighbour's (t = 0 never: B >= 16)
        return;
    u32 acc[NR * 8];
    lds_blocks<K, M, NR>(std::make_integer_sequence<int, K>{}, acc, img, B, ta, tb);
    u8 *dst = par + d.par_off;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        u32 y[8];
#pragma unroll
        for (int i = 0; i < 8; ++i)
            y[i] = acc[r * 8 + i];
        transpose8(y);
        u8 *o = dst + (u64)r * d.par_stride;
        st16(o + ta, y[0], y[1], y[2], y[3]);
        st16(o + tb, y[4], y[5], y[6], y[7]);
    }
}


// ===== sec_decode_bs_pair_kernel (SEC_SYN_PAIR: ties the direct decode, profiles/r04_syn_ab_pair.jsonl)
// ---- both phases for parity rows in BOTH groups: a wave pair (zfec(64,96), e <= 16) ------------
// A chunk whose e <= 16 present parity rows lie in both 16-row groups has no place in the one-wave
// kernel above (16 accumulator slots, one group's compile-time rows) and took the two kernels,
// which read the data once per group and send the syndromes through HBM.  Here a workgroup is two
// waves over the same span, wave g holding group g's syndromes:
//   phase 1  wave g loads, copies and transposes the present data blocks j = g mod 2 and hands
//            their bit planes to the other wave through LDS (one s_barrier per block pair), so
//            every block is read and transposed once; each wave applies its group's present
//            rows to every block, then its parity rows: scaled syndromes in its registers, and a
//            copy in LDS by global rank q;
//   phase 2  wave g solves the lost rows of 8-row groups G = g mod 2 over all e syndromes: its
//            own from registers, the other wave's from LDS.
// The syndromes never leave the CU: traffic is the decode's own (1.02x, profiles/r04_syn_pmc.json).
// Opt-in (context option SEC_SYN_PAIR = 1): on random 16-lost patterns it ties the direct decode
// (0.78 ms per GiB, 2.75-2.83 TB/s) -- its waves wait on memory 60 % of their cycles (2-block register
// ring, one barrier per block pair).  Also measured and dropped (r04_syn_ab_pair.jsonl): each wave
// running the one-wave kernel's phase 1 for its own group on an LDS DMA ring (0.85 ms: every block's
// transposes and subsets twice), and e <= 32 with 32 syndrome slots (64-72 KiB of LDS, one wave per
// SIMD: 1.62-1.66 ms against 0.80 for the two kernels).
template <int K, int M, int R0, int NRP, int J>
__device__ __forceinline__ void pd_rows(u32 (&acc)[NRP * 8], const u32 *v, uint64_t pmask)
{
    u32 lo[16], hi[16];
    subsets(v[0], v[1], v[2], v[3], lo);
    subsets(v[4], v[5], v[6], v[7], hi);
    syn_rows<K, M, R0, J>(std::make_integer_sequence<int, NRP>{}, acc, lo, hi, pmask);
}

template <int K, int M, int R0, int NRP, int D, int P>
__device__ __forceinline__ void pd_step(u32 (&acc)[NRP * 8], u32 (&ring)[D][8], const SynCtx &c,
                                        u32x4 (*planes)[2][2][64], u8 *orow0, u32 B, u32 last, bool copies, u32 lane)
{
    constexpr int G = R0 / NRP, JO = 2 * P + G, JT = 2 * P + 1 - G, JN = 2 * (P + D) + G;
    u32 x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
        x[i] = ring[P % D][i];
    if constexpr (JN < K)
        if ((c.dmask >> JN) & 1)
            load_syn_item<K, NRP, R0, JN>(ring[P % D], c);
    const bool own = (c.dmask >> JO) & 1, other = (c.dmask >> JT) & 1;
    if (own) {
        if (copies) {  // the present primary's bytes to its output row (row K-1 clamps to `last`)
            u8 *o = orow0 + (u64)JO * B;
            if constexpr (JO == K - 1) {
                st16_clamped(o, c.pa, last, x[0], x[1], x[2], x[3]);
                st16_clamped(o, c.pb, last, x[4], x[5], x[6], x[7]);
            } else {
                st16(o + c.pa, x[0], x[1], x[2], x[3]);
                st16(o + c.pb, x[4], x[5], x[6], x[7]);
            }
        }
        transpose8(x);
        planes[P & 1][G][0][lane] = u32x4{x[0], x[1], x[2], x[3]};
        planes[P & 1][G][1][lane] = u32x4{x[4], x[5], x[6], x[7]};
    }
    __syncthreads();
    if (own)
        pd_rows<K, M, R0, NRP, JO>(acc, x, c.pmask);
    __builtin_amdgcn_sched_barrier(0);
    if (other) {
        const u32x4 t0 = planes[P & 1][1 - G][0][lane], t1 = planes[P & 1][1 - G][1][lane];
        const u32 y[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
        pd_rows<K, M, R0, NRP, JT>(acc, y, c.pmask);
    }
    __builtin_amdgcn_sched_barrier(0);
}

template <int K, int M, int R0, int NRP, int D, int... Ps>
__device__ __forceinline__ void pd_steps(std::integer_sequence<int, Ps...>, u32 (&acc)[NRP * 8], u32 (&ring)[D][8],
                                         const SynCtx &c, u32x4 (*planes)[2][2][64], u8 *orow0, u32 B, u32 last,
                                         bool copies, u32 lane)
{
    (pd_step<K, M, R0, NRP, D, Ps>(acc, ring, c, planes, orow0, B, last, copies, lane), ...);
}

// parity row R0 + r of this wave's group: syndrome = its planes ^ the data's contribution, * w_q;
// kept in the accumulators and copied to LDS slot q (its rank among all present rows)
template <int K, int R0, int NRP, int r>
__device__ __forceinline__ void pd_parity(u32 (&acc)[NRP * 8], const SynCtx &c, u32x4 (*syl)[2][64], u32 lane)
{
    if (!((c.pmask >> (R0 + r)) & 1))
        return;
    u32 x[8];
    load_syn_item<K, NRP, R0, K + r>(x, c);
    transpose8(x);
    const u32 q = (u32)__builtin_popcountll(c.pmask & ((1ull << (R0 + r)) - 1ull));
    u32 y[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
        y[i] = acc[r * 8 + i] ^ x[i];
    scale_planes(y, c.wmask[q]);
#pragma unroll
    for (int i = 0; i < 8; ++i)
        acc[r * 8 + i] = y[i];
    syl[q][0][lane] = u32x4{y[0], y[1], y[2], y[3]};
    syl[q][1][lane] = u32x4{y[4], y[5], y[6], y[7]};
}

template <int K, int R0, int NRP, int... Rs>
__device__ __forceinline__ void pd_parities(std::integer_sequence<int, Rs...>, u32 (&acc)[NRP * 8], const SynCtx &c,
                                            u32x4 (*syl)[2][64], u32 lane)
{
    (pd_parity<K, R0, NRP, Rs>(acc, c, syl, lane), ...);
}

// phase 2, lost rows [G2 * NR2, G2 * NR2 + NR2): parity row PR's syndrome (own group: the
// registers; else LDS) times c[PR][lost rows]
template <int K, int M, int R0, int NRP, int NR2, int G2, int PR>
__device__ __forceinline__ void pd_solve_one(u32 (&acc2)[NR2 * 8], const u32 (&sy)[NRP * 8], const SynCtx &c,
                                             const OutCtx &o, u32x4 (*syl)[2][64], u32 lane)
{
    if (!((c.pmask >> PR) & 1))
        return;
    u32 v[8];
    if constexpr (PR >= R0 && PR < R0 + NRP) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
            v[i] = sy[(PR - R0) * 8 + i];
    } else {
        const u32 q = (u32)__builtin_popcountll(c.pmask & ((1ull << PR) - 1ull));
        const u32x4 a = syl[q][0][lane], b = syl[q][1][lane];
        v[0] = a.x, v[1] = a.y, v[2] = a.z, v[3] = a.w, v[4] = b.x, v[5] = b.y, v[6] = b.z, v[7] = b.w;
    }
    u32 lo[16], hi[16];
    subsets(v[0], v[1], v[2], v[3], lo);
    subsets(v[4], v[5], v[6], v[7], hi);
    solve_rows<K, M, G2 * NR2, NR2, PR>(std::make_integer_sequence<int, NR2>{}, acc2, lo, hi, o.lost);
}

template <int K, int M, int R0, int NRP, int NR2, int G2, int... PRs>
__device__ __forceinline__ void pd_solve_group(std::integer_sequence<int, PRs...>, const u32 (&sy)[NRP * 8],
                                               const SynCtx &c, const OutCtx &o, u32x4 (*syl)[2][64], u32 lane)
{
    if (!((o.lost >> (G2 * NR2)) & ((1ull << NR2) - 1ull)))
        return;
    u32 acc2[NR2 * 8];
#pragma unroll
    for (int i = 0; i < NR2 * 8; ++i)
        acc2[i] = 0;
    (pd_solve_one<K, M, R0, NRP, NR2, G2, PRs>(acc2, sy, c, o, syl, lane), ...);
    solve_outs<K, G2 * NR2, NR2>(std::make_integer_sequence<int, NR2>{}, acc2, o);
}

template <int K, int M, int R0, int NRP, int NR2, int... G2s>
__device__ __forceinline__ void pd_solve(std::integer_sequence<int, G2s...>, const u32 (&sy)[NRP * 8], const SynCtx &c,
                                         const OutCtx &o, u32x4 (*syl)[2][64], u32 lane)
{
    // this wave's lost-row groups: every other one, from its own index
    ((G2s % 2 == R0 / NRP ? pd_solve_group<K, M, R0, NRP, NR2, G2s>(std::make_integer_sequence<int, M - K>{}, sy, c, o,
                                                                     syl, lane)
                          : void()),
     ...);
}

// the first D own data blocks of wave R0 / NRP (blocks 2 j + g) into the ring
template <int K, int R0, int NRP, int D, int... Js>
__device__ __forceinline__ void pd_first(std::integer_sequence<int, Js...>, u32 (&ring)[D][8], const SynCtx &c)
{
    constexpr int G = R0 / NRP;
    ((((c.dmask >> (2 * Js + G)) & 1) ? load_syn_item<K, NRP, R0, 2 * Js + G>(ring[Js], c) : void()), ...);
}

template <int K, int M, int R0, int NRP, int NR2, int D>
__device__ __forceinline__ void pd_span(const u8 *__restrict__ blocks, u8 *__restrict__ out, const sec::SynDesc &d,
                                        const sec::SynSlots &sl, u32 s, bool copies, u32x4 (*planes)[2][2][64],
                                        u32x4 (*syl)[2][64])
{
    const u32 B = d.B, lane = threadIdx.x & 63;
    const SynCtx c{blocks,  sl.off,     sl.avail, sl.masks + d.wq0,     d.slot0,         min(s + 16 * lane, B - 16),
                   min(s + 1024 + 16 * lane, B - 16), s + 16 * lane, s + 1024 + 16 * lane, d.dmask, d.pmask, 0};
    u32 ring[D][8];
    pd_first<K, R0, NRP, D>(std::make_integer_sequence<int, D>{}, ring, c);
    u32 acc[NRP * 8];
#pragma unroll
    for (int i = 0; i < NRP * 8; ++i)
        acc[i] = 0;
    pd_steps<K, M, R0, NRP, D>(std::make_integer_sequence<int, K / 2>{}, acc, ring, c, planes, out + d.out_off, B,
                               d.last, copies, lane);
    pd_parities<K, R0, NRP>(std::make_integer_sequence<int, NRP>{}, acc, c, syl, lane);
    __syncthreads();  // both waves' syndromes in LDS
    const uint64_t lost = ~d.dmask & (K >= 64 ? ~0ull : (1ull << K) - 1ull);
    const OutCtx o{out + d.out_off, sl.masks + d.zq0, lost, B, d.last, d.flags & 2u ? 1u : 0u, c.pa, c.pb};
    pd_solve<K, M, R0, NRP, NR2>(std::make_integer_sequence<int, K / NR2>{}, acc, c, o, syl, lane);
}

// 128 lanes per span (tile t0), wave g = parity group g; ntail bit 0 = copy the present primaries
template <int K, int M, int NRP, int NR2, int D>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2))) void sec_decode_bs_pair_kernel(
    const u8 *__restrict__ blocks, u8 *__restrict__ out, const sec::SynDesc *__restrict__ descs,
    const sec::Tile *__restrict__ tiles, const sec::SynSlots sl)
{
    static_assert(K % 2 == 0 && M - K == 2 * NRP && K % NR2 == 0, "two parity groups over an even K");
    __shared__ u32x4 planes[2][2][2][64];  // [pair parity][wave][planes 0-3 | 4-7][lane]: 8 KiB
    __shared__ u32x4 syl[16][2][64];       // scaled syndrome q: 32 KiB (e <= 16)
    const sec::Tile tl = tiles[blockIdx.x];
    const sec::SynDesc d = descs[tl.chunk];
    if (tl.t0 >= d.B)
        return;
    const bool copies = tl.ntail & 1;
    if (threadIdx.x < 64)
        pd_span<K, M, 0, NRP, NR2, D>(blocks, out, d, sl, tl.t0, copies, planes, syl);
    else
        pd_span<K, M, NRP, NRP, NR2, D>(blocks, out, d, sl, tl.t0, copies, planes, syl);
}


// ===== sec_encode_bs_pair_kernel (SEC_BS_PAIR: -5 to -8 %, profiles/r04_bs_pair_ab.jsonl)
// ---- two row groups sharing each block's transpose (zfec(64,96)) ------------------------------
// sec_encode_bs2_kernel's two groups of 16 rows each load and transpose all K blocks (the
// transposes are 27 % of its VALU, and it runs at the VALU issue rate).  Here a workgroup is two
// waves over the SAME span, wave g computing rows [16 g, 16 g + 16): wave g loads and transposes
// only blocks j = g mod 2, hands the 8 bit planes to the other wave through LDS (double-buffered,
// one s_barrier per block pair) and takes that wave's planes of the other blocks.  Each block is
// loaded and transposed once.
template <int K, int M, int R0, int NR, int D, int P>
__device__ __forceinline__ void pair_step(u32 (&acc)[NR * 8], u32 (&ring)[D][8], u32x4 (*planes)[2][2][64],
                                          const u8 *src, u64 B, u32 pa, u32 pb, u32 valid, u32 g, u32 lane)
{
    // this wave's block of the pair: 2P + g (G = R0 / NR is g); its next-to-load own block is 2(P + D) + g
    constexpr int G = R0 / NR;
    constexpr int JO = 2 * P + G, JT = 2 * P + 1 - G;
    u32 x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
        x[i] = ring[P % D][i];
    if constexpr (2 * (P + D) + G < K)
        load_block<false>(ring[P % D], src + (u64)(2 * (P + D) + G) * B, pa, pb, valid, 2 * (P + D) + G == K - 1);
    transpose8(x);
    planes[P & 1][G][0][lane] = u32x4{x[0], x[1], x[2], x[3]};  // lanes' 16 B contiguous: no bank conflict
    planes[P & 1][G][1][lane] = u32x4{x[4], x[5], x[6], x[7]};
    __syncthreads();
    auto rows = [&](const u32 *v, auto jc) {
        constexpr int J = decltype(jc)::value;
        u32 lo[16], hi[16];
        subsets(v[0], v[1], v[2], v[3], lo);
        subsets(v[4], v[5], v[6], v[7], hi);
        block_rows<K, M, R0, J, J == 0>(std::make_integer_sequence<int, NR * 8>{}, acc, lo, hi);
    };
    auto theirs = [&](auto jc) {
        const u32x4 t0 = planes[P & 1][1 - G][0][lane], t1 = planes[P & 1][1 - G][1][lane];
        const u32 y[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
        rows(y, jc);
    };
    // the own block first (its planes are in registers), then the other wave's; block 0 (wave 0's)
    // initialises the accumulators, so wave 1 takes it first in the first pair
    // (sched_barrier: kept apart, the two blocks' subsets are never live at once)
    if constexpr (P == 0 && G == 1) {
        theirs(std::integral_constant<int, JT>{});
        __builtin_amdgcn_sched_barrier(0);
        rows(x, std::integral_constant<int, JO>{});
    } else {
        rows(x, std::integral_constant<int, JO>{});
        __builtin_amdgcn_sched_barrier(0);
        theirs(std::integral_constant<int, JT>{});
    }
    __builtin_amdgcn_sched_barrier(0);
}

template <int K, int M, int R0, int NR, int D, int... Ps>
__device__ __forceinline__ void pair_steps(std::integer_sequence<int, Ps...>, u32 (&acc)[NR * 8], u32 (&ring)[D][8],
                                           u32x4 (*planes)[2][2][64], const u8 *src, u64 B, u32 pa, u32 pb, u32 valid,
                                           u32 g, u32 lane)
{
    (pair_step<K, M, R0, NR, D, Ps>(acc, ring, planes, src, B, pa, pb, valid, g, lane), ...);
}

template <int K, int M, int R0, int NR, int D>
__device__ __forceinline__ void pair_span(const u8 *__restrict__ in, u8 *__restrict__ par, const sec::EncDesc &d,
                                          u32 s, u32x4 (*planes)[2][2][64])
{
    constexpr int G = R0 / NR;
    const u32 B = d.B, lane = threadIdx.x & 63;
    const u32 pa = min(s + 16 * lane, B - 16), pb = min(s + 1024 + 16 * lane, B - 16);
    const u8 *src = in + d.in_off;
    u32 ring[D][8];
#pragma unroll
    for (int j = 0; j < D; ++j)
        load_block<false>(ring[j], src + (u64)(2 * j + G) * B, pa, pb, d.valid, 2 * j + G == K - 1);
    u32 acc[NR * 8];
    pair_steps<K, M, R0, NR, D>(std::make_integer_sequence<int, K / 2>{}, acc, ring, planes, src, B, pa, pb, d.valid,
                                G, lane);
    u8 *dst = par + d.par_off;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        u32 y[8];
#pragma unroll
        for (int i = 0; i < 8; ++i)
            y[i] = acc[r * 8 + i];
        transpose8(y);
        u8 *o = dst + (u64)(R0 + r) * d.par_stride;
        st16(o + pa, y[0], y[1], y[2], y[3]);
        st16(o + pb, y[4], y[5], y[6], y[7]);
    }
}

// 128 lanes: wave 0 rows [0, NR), wave 1 rows [NR, 2 NR) of one span (tile t0) of one chunk.
template <int K, int M, int NR, int D>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2))) void sec_encode_bs_pair_kernel(const u8 *__restrict__ in, u8 *__restrict__ par,
                                                                 const sec::EncDesc *__restrict__ descs,
                                                                 const sec::Tile *__restrict__ tiles)
{
    static_assert(K % 2 == 0 && M - K == 2 * NR, "two row groups over an even K");
    __shared__ u32x4 planes[2][2][2][64];  // [pair parity][wave][planes 0-3 | 4-7][lane]: 8 KiB
    const sec::Tile tl = tiles[blockIdx.x];
    const sec::EncDesc d = descs[tl.chunk];
    if (tl.t0 >= d.B)
        return;
    if (threadIdx.x < 64)
        pair_span<K, M, 0, NR, D>(in, par, d, tl.t0, planes);
    else
        pair_span<K, M, NR, NR, D>(in, par, d, tl.t0, planes);
}


// ===== launcher of sec_encode_bs_lds_kernel
namespace {
template <int K, int M>
hipError_t launch_bs_lds(const u8 *in, u8 *par, const sec::EncDesc *d, const sec::Tile *t, u32 nt, hipStream_t s)
{
    void *a = nullptr, *b = nullptr;
    sec_next_launch_events(&a, &b);
    hipExtLaunchKernelGGL((sec_encode_bs_lds_kernel<K, M>), dim3(nt), dim3(256), 0, s, (hipEvent_t)a, (hipEvent_t)b, 0,
                          in, par, d, t);
    return hipGetLastError();
}
}  // namespace

uint32_t sec_bs_lds_max() { return kLdsChunk; }

int sec_launch_encode_bs_lds(int shape, const uint8_t *in, uint8_t *par, const sec::EncDesc *descs,
                             const sec::Tile *t, uint32_t ntiles, void *stream)
{
    if (ntiles == 0)
        return hipSuccess;
    hipStream_t s = (hipStream_t)stream;
    switch (shape) {
    case 0: return launch_bs_lds<10, 14>(in, par, descs, t, ntiles, s);
    case 1: return launch_bs_lds<8, 12>(in, par, descs, t, ntiles, s);
    case 2: return launch_bs_lds<16, 24>(in, par, descs, t, ntiles, s);
    case 5: return launch_bs_lds<8, 11>(in, par, descs, t, ntiles, s);
    default: return hipErrorInvalidValue;
    }
}


// ===== launcher of sec_decode_bs_pair_kernel
// SEC_PAIR_RING (build knob): own data blocks in flight per wave of the pair decode
#ifndef SEC_PAIR_RING
#define SEC_PAIR_RING 2
#endif
int sec_launch_decode_bs_pair(int shape, int e_max, const uint8_t *blocks, uint8_t *out, const sec::SynDesc *descs,
                              const sec::Tile *t, uint32_t ntiles, sec::SynSlots sl, void *stream)
{
    if (ntiles == 0)
        return hipSuccess;
    if (shape != 4 || e_max < 1 || e_max > 16)
        return hipErrorInvalidValue;
    void *a = nullptr, *b = nullptr;
    sec_next_launch_events(&a, &b);
    hipExtLaunchKernelGGL((sec_decode_bs_pair_kernel<64, 96, 16, 8, SEC_PAIR_RING>), dim3(ntiles), dim3(128), 0,
                          (hipStream_t)stream, (hipEvent_t)a, (hipEvent_t)b, 0, blocks, out, descs, t, sl);
    return hipGetLastError();
}

