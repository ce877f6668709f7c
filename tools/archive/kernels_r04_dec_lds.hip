// ARCHIVED (round 5): sec_decode_lds_kernel, the SEC_DEC_LDS opt-in of round 4.
// A/B: -28 % against the tile decode on C4 (profiles/r04_c4_lds_ab.jsonl).  Not built; kept for reference.

// ---- small chunks reassembled in LDS (C4's 64 KiB chunks) --------------------------------------
// The tiles above write a reassembled chunk as k row streams that start at zfec's block starts
// j * B (C4: 6554, so every 128-byte line at a row boundary is written in two halves by two
// waves).  Here one 256-lane workgroup per chunk of n <= 64 KiB computes the e lost rows (the
// same v_perm products over all k slots), puts the present primaries and the recovered rows into
// an LDS image of the chunk at row * B + position, and then writes the n bytes out as ONE
// contiguous run of 16-byte stores.  Lane l owns positions 16 l and 4096 + 16 l (each moved back
// to end at B when past it: it repeats a neighbour's bytes), so B <= 8192.
constexpr u32 kLdsDecChunk = 65536;

struct DecImg {
    u32x4 v[kLdsDecChunk / 16 + 4];  // the chunk, then room for row k-1's bytes past n (padlen < k <= 16)
};

// 16 bytes into the image at byte offset o, any alignment
__device__ __forceinline__ void img_put16(u8 *img, u32 o, u32x4 v)
{
    if ((o & 15) == 0) {
        *reinterpret_cast<u32x4 *>(img + o) = v;
    } else if ((o & 3) == 0) {
        u32 *p = reinterpret_cast<u32 *>(img + o);
        p[0] = v.x;
        p[1] = v.y;
        p[2] = v.z;
        p[3] = v.w;
    } else if ((o & 1) == 0) {
        uint16_t *p = reinterpret_cast<uint16_t *>(img + o);
        const u32 w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            p[2 * i] = (uint16_t)w[i];
            p[2 * i + 1] = (uint16_t)(w[i] >> 16);
        }
    } else {
        const u32 w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 16; ++i)
            img[o + i] = (u8)(w[i >> 2] >> (8 * (i & 3)));
    }
}

// 16 bytes of a slot at p of which the first `avail - p` exist (the rest read as zero)
__device__ __forceinline__ u32x4 slot16(const u8 *s, u32 p, u32 avail)
{
    if (p + 16 <= avail)
        return load16(s + p);
    u32 w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int b = 0; b < 16; ++b)
        if (p + b < avail)
            w[b >> 2] |= (u32)s[p + b] << (8 * (b & 3));
    return u32x4{w[0], w[1], w[2], w[3]};
}

template <int R>
__global__ __launch_bounds__(256) void sec_decode_lds_kernel(const u8 *__restrict__ blocks, u8 *__restrict__ out,
                                                             const sec::DecDesc *__restrict__ descs,
                                                             const sec::Tile *__restrict__ tiles,
                                                             const u32 *__restrict__ tabs, const sec::DecSlots sl)
{
    __shared__ DecImg img;
    u8 *im = reinterpret_cast<u8 *>(img.v);
    const sec::DecDesc d = descs[tiles[blockIdx.x].chunk];
    const u32 B = d.B, k = d.k, t = threadIdx.x;
    const u32 pa = min(16 * t, B - 16), pb = min(16 * t + 4096, B - 16);
    if (16 * t < B) {
        const u32 *tj = tabs + d.tab;
        const u32 tstep = d.e * sec::kTabDwords;
        u32x4 acc[R > 0 ? R : 1][2];
#pragma unroll
        for (int r = 0; r < (R > 0 ? R : 1); ++r)
            acc[r][0] = acc[r][1] = u32x4{0u, 0u, 0u, 0u};
        constexpr int KB = 8;  // slots per load batch (2 x 16 B each)
#pragma unroll 1
        for (u32 c0 = 0; c0 < k; c0 += KB) {
            u32x4 xs[KB][2];
#pragma unroll
            for (int c = 0; c < KB; ++c)
                if (c0 + c < k) {
                    const u8 *s = blocks + sl.off[d.slot0 + c0 + c];
                    const u32 av = sl.avail[d.slot0 + c0 + c];
                    xs[c][0] = slot16(s, pa, av);
                    xs[c][1] = slot16(s, pb, av);
                }
#pragma unroll
            for (int c = 0; c < KB; ++c)
                if (c0 + c < k) {
                    if constexpr (R > 0)
                        gf_mac<R, 2>(acc, xs[c], tj + (c0 + c) * tstep, nullptr);
                    const u32 orow = sl.row[d.slot0 + c0 + c];
                    if (orow != 0xFFFFFFFFu) {  // a present primary: its bytes at its row
                        img_put16(im, orow * B + pa, xs[c][0]);
                        img_put16(im, orow * B + pb, xs[c][1]);
                    }
                }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const u32 orow = sl.miss[d.slot0 + r];
            img_put16(im, orow * B + pa, acc[r][0]);
            img_put16(im, orow * B + pb, acc[r][1]);
        }
    }
    __syncthreads();
    const u32 n = (u32)d.n, nf = n / 16;
    u8 *dst = out + d.out_off;
    for (u32 v = t; v < nf; v += 256)
        store16<SEC_DEC_ST>(dst + 16 * v, img.v[v]);
    if (t < n % 16)  // the chunk's last bytes
        dst[16 * nf + t] = im[16 * nf + t];
}


// launcher
uint32_t sec_dec_lds_max() { return kLdsDecChunk; }

int sec_launch_decode_lds(int rows, const uint8_t *blocks, uint8_t *out, const sec::DecDesc *descs,
                          const sec::Tile *tiles, uint32_t ntiles, const uint32_t *tabs, sec::DecSlots sl, void *stream)
{
    if (ntiles == 0)
        return hipSuccess;
    hipStream_t s = (hipStream_t)stream;
    const dim3 g(ntiles), b(256);
    switch (rows) {
    case 0: return launch(sec_decode_lds_kernel<0>, g, b, s, blocks, out, descs, tiles, tabs, sl);
    case 1: return launch(sec_decode_lds_kernel<1>, g, b, s, blocks, out, descs, tiles, tabs, sl);
    case 2: return launch(sec_decode_lds_kernel<2>, g, b, s, blocks, out, descs, tiles, tabs, sl);
    case 3: return launch(sec_decode_lds_kernel<3>, g, b, s, blocks, out, descs, tiles, tabs, sl);
    case 4: return launch(sec_decode_lds_kernel<4>, g, b, s, blocks, out, descs, tiles, tabs, sl);
    case 5: return launch(sec_decode_lds_kernel<5>, g, b, s, blocks, out, descs, tiles, tabs, sl);
    case 6: return launch(sec_decode_lds_kernel<6>, g, b, s, blocks, out, descs, tiles, tabs, sl);
    case 7: return launch(sec_decode_lds_kernel<7>, g, b, s, blocks, out, descs, tiles, tabs, sl);
    case 8: return launch(sec_decode_lds_kernel<8>, g, b, s, blocks, out, descs, tiles, tabs, sl);
    default: return hipErrorInvalidValue;
    }
}

