// yavo_inflate.hip -- PNG decoding on the GPU for a batch of frames: the device half of cv::imread(path, 0)
// (src/LoopHandler.cc:919) for 8-bit grey, non-interlaced PNGs (every KITTI frame; the reference's own
// tests/epilines.png).  The host only reads the files and gathers each image's IDAT payload (its zlib stream); the
// GPU inflates it (RFC 1950 / 1951) and undoes the scanline filters (PNG filter method 0).
//
// inflate: one 64-lane wave per image.  Huffman decoding is sequential, so the decoder state (bit buffer, stream
// position, output position) is wave-uniform and lives in SGPRs; lookups go to tables in the wave's LDS (a fast table
// per code indexed by the next 10 / 8 stream bits, canonical decoding for longer codes).  Output bytes go to a 32 KB
// LDS ring (the deflate window, which back-references read) and every completed 4 KB of it is streamed to HBM by all
// 64 lanes.  Length / distance copies use the lanes: byte j of a match of length L at distance D is the window byte
// op - D + (j mod D), so each LDS read + write moves up to 64 bytes whatever D is.  The images of a batch decode
// concurrently; the per-symbol latency of each wave sets the rate.  The Adler-32 trailer is not checked.
//
// unfilter: one wave per image, lane l owning row 64 b + l of band b.  Row r needs row r - 1 (Up / Average / Paeth),
// so lane l runs one step behind lane l - 1: at step t it undoes the 4-byte group t - l of its row, and the same
// group of the row above, made by lane l - 1 at step t - 1, arrives by one DPP wave shift.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "yavo_internal.h"

namespace yavo {
namespace png {

constexpr int kRing = 32768;  // deflate window
constexpr int kRingMask = kRing - 1;
constexpr int kFlush = 4096;  // ring bytes streamed to HBM at once
constexpr int kLitBits = 10, kDistBits = 8;

struct Table {
    uint16_t cnt[16];   // codes per length
    uint16_t offs[16];  // first index of each length in sym
    uint16_t next[16];  // first canonical code of each length
    uint16_t sym[288];  // symbols ordered by (length, symbol)
};

struct Lds {
    uint8_t ring[kRing];
    uint16_t lit_fast[1 << kLitBits];  // (symbol << 4) | length; 0: the code is longer than kLitBits
    uint16_t dist_fast[1 << kDistBits];
    Table lit, dist;
    uint8_t lens[320];  // code lengths: litlen [0, 288), distance [288, 320); the code-length code in [0, 19)
    uint8_t cl[20];
};

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// bit reader over a 4-B aligned stream, LSB first (RFC 1951 3.1.1)
struct Bits {
    const uint32_t* src;
    uint32_t nwords, wp;  // words in the stream, next word to load
    uint64_t bb;          // bit buffer
    uint32_t nb;          // valid bits in bb
    uint32_t over;        // words read past the end (zeros)
    __device__ __forceinline__ void refill() {
        if (nb <= 32) {
            uint32_t w = 0;
            if (wp < nwords) w = src[wp];
            else ++over;
            ++wp;
            bb |= (uint64_t)w << nb;
            nb += 32;
        }
    }
    __device__ __forceinline__ uint32_t peek(uint32_t n) const { return (uint32_t)bb & ((1u << n) - 1u); }
    __device__ __forceinline__ void drop(uint32_t n) {
        bb >>= n;
        nb -= n;
    }
    __device__ __forceinline__ uint32_t get(uint32_t n) {  // n <= 16
        refill();
        const uint32_t v = peek(n);
        drop(n);
        return v;
    }
};

// Canonical Huffman tables from the code lengths lens[0, n) in LDS (RFC 1951 3.2.2): counts, the symbols sorted by
// (length, symbol), and the fast table: entry (reversed code + k 2^len) = (symbol << 4) | len for len <= fast_bits.
// Lane-parallel over the symbols: counts and per-length ranks from ballots (wave-uniform running totals in SGPRs),
// fast-table replicas written by the lanes.  Returns false on an over-subscribed code (incomplete codes are
// accepted, as zlib's inflate does).
__device__ bool build_table(const uint8_t* lens, int n, Table& T, uint16_t* fast, int fast_bits) {
    const int lane = threadIdx.x & 63;
    const uint64_t below = (1ull << lane) - 1ull;
    for (int i = lane; i < (1 << fast_bits); i += 64) fast[i] = 0;
    uint32_t c[16];
#pragma unroll
    for (int l = 0; l < 16; ++l) c[l] = 0;
    for (int s0 = 0; s0 < n; s0 += 64) {
        const int l = s0 + lane < n ? (int)lens[s0 + lane] : 0;
#pragma unroll
        for (int len = 1; len < 16; ++len) c[len] += (uint32_t)__popcll(__ballot(l == len));
    }
    int left = 1;
    uint32_t off[16], nxt[16], code = 0;
    off[0] = nxt[0] = 0;
#pragma unroll
    for (int l = 1; l < 16; ++l) {
        left = (left << 1) - (int)c[l];
        code = (code + c[l - 1]) << 1;
        nxt[l] = code;
        off[l] = l == 1 ? 0 : off[l - 1] + c[l - 1];
    }
    if (left < 0) return false;
    if (lane == 0) {
#pragma unroll
        for (int l = 0; l < 16; ++l) {
            T.cnt[l] = (uint16_t)c[l];
            T.offs[l] = (uint16_t)off[l];
            T.next[l] = (uint16_t)nxt[l];
        }
    }
    __builtin_amdgcn_wave_barrier();
    uint32_t run[16];
#pragma unroll
    for (int l = 0; l < 16; ++l) run[l] = 0;
    for (int s0 = 0; s0 < n; s0 += 64) {
        const int s = s0 + lane;
        const int l = s < n ? (int)lens[s] : 0;
        uint32_t idx = 0;
#pragma unroll
        for (int len = 1; len < 16; ++len) {
            const uint64_t m = __ballot(l == len);
            if (l == len) idx = run[len] + (uint32_t)__popcll(m & below);
            run[len] += (uint32_t)__popcll(m);
        }
        if (l) {
            T.sym[T.offs[l] + idx] = (uint16_t)s;
            if (l <= fast_bits) {
                const uint32_t cd = (uint32_t)T.next[l] + idx;
                const uint32_t rev = __builtin_bitreverse32(cd) >> (32 - l);
                const uint16_t e = (uint16_t)((s << 4) | l);
                for (uint32_t k = 0; k < (1u << (fast_bits - l)); ++k) fast[rev + (k << l)] = e;
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    return true;
}

// one symbol: the fast table, else canonical decoding bit by bit (RFC 1951 3.2.2; zlib's puff.c decode())
__device__ __forceinline__ int decode_sym(Bits& br, const uint16_t* fast, int fast_bits, const Table& T) {
    br.refill();
    const uint32_t e = uni(fast[br.peek(fast_bits)]);
    if (e) {
        br.drop(e & 15u);
        return (int)(e >> 4);
    }
    int code = 0, first = 0, index = 0;
    for (int len = 1; len < 16; ++len) {
        code |= (int)(br.bb & 1u);
        br.drop(1);
        const int count = (int)uni(T.cnt[len]);
        if (code - count < first) return (int)uni(T.sym[index + (code - first)]);
        index += count;
        first += count;
        first <<= 1;
        code <<= 1;
    }
    return -1;
}

// ring bytes [from, to) of the output to HBM (from a multiple of 16)
__device__ void flush(const Lds& S, uint8_t* out, uint32_t from, uint32_t to) {
    const int lane = threadIdx.x & 63;
    for (uint32_t p = from + 16u * lane; p < to; p += 1024u) {
        if (p + 16u <= to) {
            const uint4 v = *reinterpret_cast<const uint4*>(&S.ring[p & kRingMask]);
            __builtin_memcpy(out + p, &v, 16);
        } else {
            for (uint32_t q = p; q < to; ++q) out[q] = S.ring[q & kRingMask];
        }
    }
}

__constant__ uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                      31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                      2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t kDistBase[30] = {1,    2,    3,    4,    5,    7,     9,     13,    17,  25,
                                       33,   49,   65,   97,   129,  193,   257,   385,   513, 769,
                                       1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6,
                                       6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// image i: zlib stream at src + off[i] (4-B aligned), len[i] bytes -> out_len bytes at out + i * out_pitch
__global__ __launch_bounds__(64) void inflate_kernel(const uint8_t* __restrict__ src, const int64_t* __restrict__ off,
                                                     const int32_t* __restrict__ len, uint8_t* __restrict__ out,
                                                     int64_t out_pitch, uint32_t out_len, int32_t* __restrict__ status) {
    extern __shared__ __align__(16) uint8_t lds_raw[];
    Lds& S = *reinterpret_cast<Lds*>(lds_raw);
    const int img = blockIdx.x;
    const int lane = threadIdx.x & 63;
    uint8_t* dst = out + (int64_t)img * out_pitch;
    Bits br;
    br.src = reinterpret_cast<const uint32_t*>(src + off[img]);
    br.nwords = (uint32_t)(len[img] + 3) / 4;
    br.wp = 0;
    br.bb = 0;
    br.nb = 0;
    br.over = 0;
    int32_t st = kPngOk;
    uint32_t op = 0, flushed = 0;
    // zlib header (RFC 1950): CM 8, CINFO <= 7, no preset dictionary, FCHECK
    {
        const uint32_t cmf = br.get(8), flg = br.get(8);
        if ((cmf & 15u) != 8u || (cmf >> 4) > 7u || (flg & 32u) || ((cmf << 8) | flg) % 31u) st = kPngErrHeader;
    }
    bool last = false;
    while (st == kPngOk && !last) {
        if (br.over > 2) {  // a damaged stream decoding zeros past its end: every block then fails or ends, but stop
            st = kPngErrShort;
            break;
        }
        last = br.get(1) != 0;
        const uint32_t type = br.get(2);
        if (type == 0) {
            // stored block: byte-align, LEN, NLEN, LEN raw bytes
            br.drop(br.nb & 7u);
            const uint32_t n = br.get(16), nn = br.get(16);
            if ((n ^ 0xFFFFu) != nn) {
                st = kPngErrBlock;
                break;
            }
            if (op + n > out_len) {
                st = kPngErrOverrun;
                break;
            }
            for (uint32_t k = 0; k < n; ++k) {
                const uint32_t v = br.get(8);
                if (lane == 0) S.ring[(op + k) & kRingMask] = (uint8_t)v;
                __builtin_amdgcn_wave_barrier();
                if (((op + k + 1) & (kFlush - 1)) == 0) {
                    flush(S, dst, flushed, op + k + 1);
                    flushed = op + k + 1;
                    __builtin_amdgcn_wave_barrier();
                }
            }
            op += n;
            continue;
        }
        if (type == 3) {
            st = kPngErrBlock;
            break;
        }
        if (type == 1) {
            // fixed codes (RFC 1951 3.2.6)
            for (int s = lane; s < 320; s += 64) S.lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : 5;
            __builtin_amdgcn_wave_barrier();
        } else {
            const uint32_t hlit = br.get(5) + 257, hdist = br.get(5) + 1, hclen = br.get(4) + 4;
            if (hlit > 286 || hdist > 30) {
                st = kPngErrBlock;
                break;
            }
            if (lane < 20) S.cl[lane] = 0;
            __builtin_amdgcn_wave_barrier();
            for (uint32_t k = 0; k < hclen; ++k) {
                const uint32_t v = br.get(3);
                if (lane == 0) S.cl[kClOrder[k]] = (uint8_t)v;
            }
            __builtin_amdgcn_wave_barrier();
            // the code-length code: its table in dist_fast / dist (7-bit codes)
            if (!build_table(S.cl, 19, S.dist, S.dist_fast, kDistBits)) {
                st = kPngErrCode;
                break;
            }
            // hlit + hdist code lengths, litlen into lens[0, hlit), distance into lens[288, 288 + hdist)
            for (int s = lane; s < 320; s += 64) S.lens[s] = 0;
            __builtin_amdgcn_wave_barrier();
            uint32_t k = 0, prevlen = 0;
            const uint32_t total = hlit + hdist;
            while (k < total) {
                const int sym = decode_sym(br, S.dist_fast, kDistBits, S.dist);
                uint32_t rep = 1, val = (uint32_t)sym;
                if (sym < 0 || sym > 18) {
                    st = kPngErrCode;
                    break;
                }
                if (sym == 16) {
                    if (k == 0) {
                        st = kPngErrCode;
                        break;
                    }
                    val = prevlen;
                    rep = 3 + br.get(2);
                } else if (sym == 17) {
                    val = 0;
                    rep = 3 + br.get(3);
                } else if (sym == 18) {
                    val = 0;
                    rep = 11 + br.get(7);
                }
                if (k + rep > total) {
                    st = kPngErrCode;
                    break;
                }
                for (uint32_t q = lane; q < rep; q += 64) {
                    const uint32_t idx = k + q;
                    S.lens[idx < hlit ? idx : 288 + (idx - hlit)] = (uint8_t)val;
                }
                prevlen = val;
                k += rep;
            }
            if (st != kPngOk) break;
            __builtin_amdgcn_wave_barrier();
            if (uni(S.lens[256]) == 0) {  // no end-of-block code
                st = kPngErrCode;
                break;
            }
        }
        if (!build_table(S.lens, 288, S.lit, S.lit_fast, kLitBits) ||
            !build_table(S.lens + 288, 30, S.dist, S.dist_fast, kDistBits)) {
            st = kPngErrCode;
            break;
        }
        // the block's symbols
        while (true) {
            const int sym = decode_sym(br, S.lit_fast, kLitBits, S.lit);
            if (sym < 256) {
                if (sym < 0 || op >= out_len) {
                    st = sym < 0 ? kPngErrCode : kPngErrOverrun;
                    break;
                }
                if (lane == 0) S.ring[op & kRingMask] = (uint8_t)sym;
                ++op;
            } else if (sym == 256) {
                break;
            } else {
                const int li = sym - 257;
                if (li >= 29) {
                    st = kPngErrCode;
                    break;
                }
                const uint32_t L = kLenBase[li] + br.get(kLenExtra[li]);
                const int ds = decode_sym(br, S.dist_fast, kDistBits, S.dist);
                if (ds < 0 || ds >= 30) {
                    st = kPngErrCode;
                    break;
                }
                const uint32_t D = kDistBase[ds] + br.get(kDistExtra[ds]);
                if (D > op || op + L > out_len) {
                    st = D > op ? kPngErrCode : kPngErrOverrun;
                    break;
                }
                // byte j of the match = window byte op - D + (j mod D); 64 bytes per pass, every read before the writes
                __builtin_amdgcn_wave_barrier();
                for (uint32_t j0 = 0; j0 < L; j0 += 64) {
                    const uint32_t j = j0 + lane;
                    uint32_t v = 0;
                    if (j < L) v = S.ring[(op - D + (j % D)) & kRingMask];
                    __builtin_amdgcn_wave_barrier();
                    if (j < L) S.ring[(op + j) & kRingMask] = (uint8_t)v;
                    __builtin_amdgcn_wave_barrier();
                }
                op += L;
            }
            if ((op & ~(uint32_t)(kFlush - 1)) != flushed) {
                const uint32_t to = op & ~(uint32_t)(kFlush - 1);
                __builtin_amdgcn_wave_barrier();
                flush(S, dst, flushed, to);
                flushed = to;
                __builtin_amdgcn_wave_barrier();
            }
        }
    }
    if (st == kPngOk && br.over > 1) st = kPngErrShort;  // decoding ran past the stream (beyond the look-ahead word)
    if (st == kPngOk && op != out_len) st = kPngErrShort;
    __builtin_amdgcn_wave_barrier();
    if (st == kPngOk) flush(S, dst, flushed, op);
    if (lane == 0) status[img] = st;
}

__device__ __forceinline__ uint32_t byte_of(uint32_t v, int k) { return (v >> (8 * k)) & 0xFFu; }

// PNG scanline filters (filter method 0) of 8-bit grey rows: raw rows of 1 + W bytes (filter type first) -> rows of W
// bytes at dst + i * dst_pitch with row stride dst_stride.  Wavefront over rows (see the file comment).
__global__ __launch_bounds__(64) void unfilter_kernel(const uint8_t* __restrict__ raw, int64_t raw_pitch, int H, int W,
                                                      uint8_t* __restrict__ dst, int64_t dst_pitch, int dst_stride,
                                                      int32_t* __restrict__ status) {
    const int img = blockIdx.x;
    const int lane = threadIdx.x & 63;
    if (status[img] != kPngOk) return;  // wave-uniform
    const uint8_t* rimg = raw + (int64_t)img * raw_pitch;
    uint8_t* dimg = dst + (int64_t)img * dst_pitch;
    const int G = (W + 3) >> 2;  // 4-byte groups per row
    int bad = 0;
    for (int r0 = 0; r0 < H; r0 += 64) {
        const int r = r0 + lane;
        const bool row_ok = r < H;
        const uint8_t* rr = rimg + (int64_t)(row_ok ? r : 0) * (W + 1);
        const int f = row_ok ? rr[0] : 0;
        bad |= f > 4 ? 1 : 0;
        uint32_t out = 0;       // this lane's group of the last step (DPP source)
        uint32_t left = 0;      // this row's byte before the current group ("a" of its first byte)
        uint32_t upleft = 0;    // the row above's byte before the current group ("c" of its first byte)
        for (int t = 0; t < G + 63; ++t) {
            const int g = t - lane;
            // the row above's group g: lane - 1's output of the last step (wave_shr:1), for lane 0 row r0 - 1 from HBM
            uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)out, 0x138, 0xf, 0xf, false);
            const bool active = row_ok && g >= 0 && g < G;
            if (lane == 0) {
                up = 0;
                if (active && r0 > 0) {
                    const uint8_t* pr = dimg + (int64_t)(r0 - 1) * dst_stride + 4 * g;
                    const int nb = min(4, W - 4 * g);
                    for (int k = 0; k < nb; ++k) up |= (uint32_t)pr[k] << (8 * k);
                }
            }
            if (r == 0) up = 0;  // nothing above the first row
            if (active) {
                const int nb = min(4, W - 4 * g);
                uint32_t x;
                __builtin_memcpy(&x, rr + 1 + 4 * g, 4);  // the raw buffer is padded: the last group may over-read
                uint32_t a = left, c = upleft, o = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t b = byte_of(up, k);
                    const int pa = abs((int)b - (int)c), pb = abs((int)a - (int)c), pc = abs((int)a + (int)b - 2 * (int)c);
                    const uint32_t paeth = (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
                    const uint32_t pred = f == 0 ? 0u : f == 1 ? a : f == 2 ? b : f == 3 ? ((a + b) >> 1) : paeth;
                    const uint32_t v = (byte_of(x, k) + pred) & 0xFFu;
                    o |= v << (8 * k);
                    a = v;
                    c = b;
                }
                left = a;
                upleft = c;
                uint8_t* po = dimg + (int64_t)r * dst_stride + 4 * g;
                if (nb == 4) __builtin_memcpy(po, &o, 4);
                else
                    for (int k = 0; k < nb; ++k) po[k] = (uint8_t)(o >> (8 * k));
                out = o;
            } else {
                out = 0;
            }
        }
    }
    const uint64_t any_bad = __ballot(bad != 0);
    if (lane == 0 && any_bad) status[img] = kPngErrFilter;
}

}  // namespace png

void launch_png_inflate(const uint8_t* src, const int64_t* off, const int32_t* len, int n, uint8_t* out,
                        int64_t out_pitch, uint32_t out_len, int32_t* status, hipStream_t s) {
    hipLaunchKernelGGL(png::inflate_kernel, dim3(n), dim3(64), sizeof(png::Lds), s, src, off, len, out, out_pitch,
                       out_len, status);
}

void launch_png_unfilter(const uint8_t* raw, int64_t raw_pitch, int n, int H, int W, uint8_t* dst, int64_t dst_pitch,
                         int dst_stride, int32_t* status, hipStream_t s) {
    hipLaunchKernelGGL(png::unfilter_kernel, dim3(n), dim3(64), 0, s, raw, raw_pitch, H, W, dst, dst_pitch, dst_stride,
                       status);
}

}  // namespace yavo
