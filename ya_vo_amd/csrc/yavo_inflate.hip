// yavo_inflate.hip -- PNG decoding on the GPU for a batch of frames: the device half of cv::imread(path, 0)
// (src/LoopHandler.cc:919) for 8-bit grey, non-interlaced PNGs (every KITTI frame; the reference's own
// tests/epilines.png).  The host only reads the files and gathers each image's IDAT payload (its zlib stream); the
// GPU inflates it (RFC 1950 / 1951) and undoes the scanline filters (PNG filter method 0).
//
// inflate: one 64-lane wave per image, and the 64 lanes decode ONE deflate block together.  Huffman codes
// self-synchronise: a decoder started at an arbitrary bit falls onto the true token boundaries within a few tokens
// (measured on cv::imwrite KITTI-size frames: 34 bits on average, 99% within 167).  So a chunk of the block's bits is
// cut into 64 segments of `seg` bits; lane k decodes segment k, starting kLead bits early to synchronise, and records
// where its last token ends.  A lane whose start differs from where its left neighbour ended re-decodes from there
// (rarely needed twice); lane 0 starts at the true position, so the fixed point is the true token sequence.  Then a
// prefix sum over the lanes' output counts places every lane's output, a second decode of the segment writes the
// literals into the wave's LDS output ring and lists the (length, distance) matches, and the wave copies the matches
// in stream order, 64 bytes per pass (byte j of a match = output byte op - D + (j mod D)).  The block's end-of-block
// token ends the chunk early.  Block headers are parsed wave-uniformly; the dynamic code lengths use the same
// lane-parallel decoder (repeat code 16 is a distance-1 match).  Completed 16-byte groups of the ring are streamed to
// HBM after every chunk; matches reaching further back than the 8 KB ring read the already-written output.
//
// integrity, as libpng / zlib check it for cv::imread: every IDAT chunk's CRC-32 (over its type and data) is computed
// by the gather kernel (a wave per chunk, slice-by-8 tables in LDS per lane segment, the lanes' CRCs joined by the
// GF(2) combination rule), and the Adler-32 of the inflated bytes by the unfilter kernel (per lane sum d and sum i d
// by v_dot4, one 64-bit reduction), checked against the zlib trailer the inflate kernel reads after the final
// block.  A failing image gets its own status code and a zero-filled output.
//
// unfilter: one wave per image, lane l owning row 64 b + l of band b.  Row r needs row r - 1 (Up / Average / Paeth),
// so lane l runs one step behind lane l - 1: at step t it undoes the 4-byte group t - l of its row, and the same
// group of the row above, made by lane l - 1 at step t - 1, arrives by one DPP wave shift.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "yavo_internal.h"

namespace yavo {
namespace png {

// LDS per wave <= 17.5 KB: nine waves per CU, so a step's 2 x 1024 + 2 images are resident at once
constexpr int kRing = 8192;  // LDS output ring
constexpr uint32_t kRingMask = kRing - 1;
constexpr int kLitBits = 10, kDistBits = 8, kClBits = 7;  // fast-table index widths
constexpr uint32_t kSegMax = 512, kSegMin = 32;          // bits per lane per chunk
constexpr uint32_t kLead = 256;                          // synchronisation lead-in, bits
constexpr int kStageWords = (2 * kSegMax + 8 + 31) / 32 * 32;  // the chunk's stream words (+ look-ahead), whole rows
constexpr int kMaxMatch = 256;                           // matches listed per chunk
constexpr uint32_t kCap = kRing - 64;                    // output bytes per chunk (the ring keeps the unflushed tail)
// kSegMin: lane 0's segment alone always fits (<= 16 tokens start in 32 bits, <= 258 bytes each)
static_assert(16 * 258 <= (int)kCap && 16 <= kMaxMatch, "minimum segment");

struct alignas(8) LenInfo {  // one ds_read_b64
    uint16_t next;  // first canonical code of the length
    uint16_t cnt;   // codes of the length
    uint16_t offs;  // index of its first symbol in sym
    uint16_t pad;
};

template <int NS>
struct Table {
    LenInfo len[16];
    uint16_t sym[NS];  // symbols ordered by (length, symbol)
};

struct Lds {
    alignas(16) uint8_t ring[kRing];
    alignas(16) uint32_t stage[kStageWords];
    alignas(16) union {
        uint16_t lit_fast[1 << kLitBits];  // (symbol << 4) | length; 0: longer than kLitBits (or no code)
        struct {
            uint8_t lens[320];  // code lengths while a block header is read: litlen [0, 288), distance [288, 320)
            uint8_t cl[20];     // the code-length code's lengths
        } h;                    // (the litlen table is built last, after every read of lens)
    } u;
    alignas(16) uint16_t dist_fast[1 << kDistBits];  // distance codes; the code-length code while lengths are read
    uint32_t mdst[kMaxMatch];                        // the chunk's matches: output position,
    uint32_t mld[kMaxMatch];                         // (length << 16) | distance
    Table<288> lit;
    Table<32> dist;  // distance codes (30) or the code-length code (19)
};
static_assert(sizeof(Lds) <= 17920, "nine waves per CU (2304 resident images on 256 CUs)");

// stage word i's slot: XOR-swizzled within each 32-word row, so that the lanes' segments (seg / 32 words apart) fall
// on different LDS banks (ds_read_b32 banks = dword index mod 32; unswizzled, 512-bit segments were 16-way conflicts)
__device__ __forceinline__ uint32_t sw(uint32_t i) { return i ^ ((i >> 5) & 31u); }

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint32_t lane_of(uint32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

// ---- CRC-32 (ISO-HDLC: reflected polynomial 0xEDB88320, init and final XOR ~0; the PNG chunk CRC) ----
constexpr uint32_t kCrcPoly = 0xEDB88320u;
struct CrcTables {
    uint32_t t[8][256];  // slice-by-8: t[k][b] = the CRC contribution of byte b followed by k zero bytes
};
constexpr CrcTables make_crc_tables() {
    CrcTables r{};
    for (uint32_t b = 0; b < 256; ++b) {
        uint32_t c = b;
        for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ kCrcPoly : c >> 1;
        r.t[0][b] = c;
    }
    for (int k = 1; k < 8; ++k)
        for (uint32_t b = 0; b < 256; ++b) r.t[k][b] = (r.t[k - 1][b] >> 8) ^ r.t[0][r.t[k - 1][b] & 0xFFu];
    return r;
}
__constant__ CrcTables kCrcTab = make_crc_tables();

// a(x) b(x) mod P(x) in the reflected representation (bit 31 = x^0)
__device__ __forceinline__ uint32_t crc_multmodp(uint32_t a, uint32_t b) {
    uint32_t p = 0;
#pragma unroll
    for (int k = 31; k >= 0; --k) {
        p ^= (a >> k) & 1u ? b : 0u;
        b = (b & 1u) ? (b >> 1) ^ kCrcPoly : b >> 1;
    }
    return p;
}
// x^(8 n) mod P: square-and-multiply over the bits of n, from x^8
__device__ uint32_t crc_x8n(uint32_t n) {
    uint32_t p = 1u << 31;     // x^0
    uint32_t sq = 1u << 23;    // x^8
    while (n) {
        if (n & 1u) p = crc_multmodp(sq, p);
        sq = crc_multmodp(sq, sq);
        n >>= 1;
    }
    return p;
}
// CRC of A followed by B (len_b bytes) from CRC(A) and CRC(B) (the zlib crc32_combine rule)
__device__ __forceinline__ uint32_t crc_combine(uint32_t ca, uint32_t cb, uint32_t len_b) {
    return crc_multmodp(crc_x8n(len_b), ca) ^ cb;
}

// wave-uniform bit reader over a 4-B aligned stream, LSB first (RFC 1951 3.1.1); block headers only
struct Bits {
    const uint32_t* src;
    uint32_t nwords;
    uint32_t pos;  // absolute bit position
    __device__ __forceinline__ uint32_t word(uint32_t w) const { return w < nwords ? src[w] : 0u; }
    __device__ __forceinline__ uint32_t get(uint32_t n) {  // n <= 16
        const uint32_t w = pos >> 5, sh = pos & 31u;
        const uint64_t x = (((uint64_t)word(w + 1) << 32) | word(w)) >> sh;
        pos += n;
        return (uint32_t)x & ((1u << n) - 1u);
    }
};

// Canonical Huffman tables from the code lengths lens[0, n) (RFC 1951 3.2.2): counts, first codes, the symbols sorted
// by (length, symbol) for codes longer than the fast table, and the fast table of 2^F entries (entry i: the code whose
// bits, first bit lowest, are a prefix of i).  Ranks come from ballots; the fast table is built by doubling: the table
// for codes of <= l - 1 bits is copied once to fill 2^l entries, then the l-bit codes are placed.  Returns false on
// an over-subscribed code (incomplete codes are accepted, as zlib's inflate does).
template <int NS>
__device__ bool build_table(const uint8_t* lens, int n, Table<NS>& T, uint16_t* fast, int F) {
    const int lane = threadIdx.x & 63;
    const uint64_t below = (1ull << lane) - 1ull;
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
        T.len[0] = LenInfo{0, 0, 0, 0};
#pragma unroll
        for (int l = 1; l < 16; ++l) T.len[l] = LenInfo{(uint16_t)nxt[l], (uint16_t)c[l], (uint16_t)off[l], 0};
    }
    __builtin_amdgcn_wave_barrier();
    constexpr int G = 5;  // n <= 320
    uint32_t gl[G], gr[G], ge[G];
    uint32_t run[16];
#pragma unroll
    for (int l = 0; l < 16; ++l) run[l] = 0;
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int s = 64 * g + lane;
        const int l = s < n ? (int)lens[s] : 0;
        uint32_t idx = 0;
#pragma unroll
        for (int len = 1; len < 16; ++len) {
            const uint64_t m = __ballot(l == len);
            if (l == len) idx = run[len] + (uint32_t)__popcll(m & below);
            run[len] += (uint32_t)__popcll(m);
        }
        gl[g] = (uint32_t)l;
        gr[g] = 0;
        ge[g] = ((uint32_t)s << 4) | (uint32_t)l;
        if (l) {  // per-lane length: the LDS copies of off / nxt
            const LenInfo li = T.len[l];
            T.sym[li.offs + idx] = (uint16_t)s;
            gr[g] = __builtin_bitreverse32((uint32_t)li.next + idx) >> (32 - l);
        }
    }
    if (lane < 2) fast[lane] = 0;
    __builtin_amdgcn_wave_barrier();
    for (int l = 1; l <= F; ++l) {
        if (l > 1) {  // entries [h, 2h) = entries [0, h)
            const int h = 1 << (l - 1);
            if (h < 8) {
                if (lane < h) fast[h + lane] = fast[lane];
            } else {
                uint4* f4 = reinterpret_cast<uint4*>(fast);
                for (int i = lane; i < h / 8; i += 64) f4[h / 8 + i] = f4[i];
            }
            __builtin_amdgcn_wave_barrier();
        }
#pragma unroll
        for (int g = 0; g < G; ++g)
            if (gl[g] == (uint32_t)l) fast[gr[g]] = (uint16_t)ge[g];
        __builtin_amdgcn_wave_barrier();
    }
    return true;
}

// a code longer than the fast table (F bits): canonical decoding from the first 15 stream bits (bit 0 first).  The
// length table entries F+1..15 are all read first (one LDS round trip), every candidate length is tested without a
// branch (the code is prefix free: at most one matches), then the symbol is read (a second round trip).
template <int F, int NS>
__device__ __forceinline__ bool slow_code(const Table<NS>& T, uint32_t bits, uint32_t& len, uint32_t& sym) {
    const uint32_t rev = __builtin_bitreverse32(bits) >> 17;
    uint2 li[15 - F];
#pragma unroll
    for (int l = F + 1; l < 16; ++l) li[l - F - 1] = *reinterpret_cast<const uint2*>(&T.len[l]);
    uint32_t found = 0, idx = 0;
#pragma unroll
    for (int l = F + 1; l < 16; ++l) {
        const uint2 v = li[l - F - 1];
        const uint32_t i = (rev >> (15 - l)) - (v.x & 0xFFFFu);
        const bool hit = i < (v.x >> 16);
        found = hit ? (uint32_t)l : found;
        idx = hit ? (v.y & 0xFFFFu) + i : idx;
    }
    if (!found) return false;
    len = found;
    sym = T.sym[idx];
    return true;
}

__constant__ uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

enum : uint32_t { kLit = 0, kMatch = 1, kFill = 2, kEob = 3, kErr = 4 };

// One token at bit p of the staged chunk (stage[0] = stream word w0): a literal (a = byte), a match (a = length,
// b = distance), a fill of a zero code lengths (code-length codes 17 / 18) or end of block; nbits = its size.
// CL: the code-length alphabet (RFC 1951 3.2.7), code 16 = distance-1 match of 3..6.
template <bool CL>
__device__ __forceinline__ uint32_t decode_tok(const Lds& S, uint32_t w0, uint32_t p, uint32_t& nbits, uint32_t& a,
                                               uint32_t& b) {
    const uint32_t i = (p >> 5) - w0, sh = p & 31u;
    const uint32_t x0 = S.stage[sw(i)], x1 = S.stage[sw(i + 1)], x2 = S.stage[sw(i + 2)];
    const uint32_t lo = __builtin_amdgcn_alignbit(x1, x0, sh);
    const uint32_t hi = __builtin_amdgcn_alignbit(x2, x1, sh);
    if (CL) {
        const uint32_t e = S.dist_fast[lo & ((1u << kClBits) - 1u)];
        if (!e) return kErr;
        const uint32_t len = e & 15u, sym = e >> 4;
        if (sym < 16) {
            a = sym;
            nbits = len;
            return kLit;
        }
        if (sym == 16) {
            a = 3 + ((lo >> len) & 3u);
            b = 1;
            nbits = len + 2;
            return kMatch;
        }
        const uint32_t xb = sym == 17 ? 3u : 7u;
        a = (sym == 17 ? 3u : 11u) + ((lo >> len) & ((1u << xb) - 1u));
        nbits = len + xb;
        return kFill;
    }
    uint32_t e = S.u.lit_fast[lo & ((1u << kLitBits) - 1u)], len, sym;
    if (e) {
        len = e & 15u;
        sym = e >> 4;
    } else if (!slow_code<kLitBits>(S.lit, lo, len, sym)) {
        return kErr;
    }
    if (sym < 256) {
        a = sym;
        nbits = len;
        return kLit;
    }
    if (sym == 256) {
        nbits = len;
        return kEob;
    }
    const uint32_t li = sym - 257;
    if (li >= 29) return kErr;
    // length base / extra bits (RFC 1951 3.2.5) from the symbol: 3..10 plain, then 4 per extra-bit count, 258
    uint32_t le = 0, lb = li + 3;
    if (li == 28) {
        lb = 258;
    } else if (li >= 8) {
        le = (li >> 2) - 1;
        lb = ((4u | (li & 3u)) << le) + 3;
    }
    a = lb + ((lo >> len) & ((1u << le) - 1u));
    const uint32_t q = len + le;  // <= 20
    const uint32_t dv = (uint32_t)((((uint64_t)hi << 32) | lo) >> q);
    uint32_t e2 = S.dist_fast[dv & ((1u << kDistBits) - 1u)], dl, ds;
    if (e2) {
        dl = e2 & 15u;
        ds = e2 >> 4;
    } else if (!slow_code<kDistBits>(S.dist, dv, dl, ds)) {
        return kErr;
    }
    if (ds >= 30) return kErr;
    uint32_t de = 0, db = ds + 1;
    if (ds >= 4) {
        de = (ds >> 1) - 1;
        db = ((2u | (ds & 1u)) << de) + 1;
    }
    b = db + ((dv >> dl) & ((1u << de) - 1u));  // dl + de <= 28
    nbits = q + dl + de;                        // <= 48
    return kMatch;
}

// tokens from p while p < to: output bytes, matches, stop (1 end of block, 2 invalid code)
template <bool CL>
__device__ __forceinline__ void count_pass(const Lds& S, uint32_t w0, uint32_t& p, uint32_t to, uint32_t& cnt,
                                           uint32_t& nmt, uint32_t& stop) {
    cnt = 0;
    nmt = 0;
    stop = 0;
    while (p < to) {
        uint32_t nb = 0, a = 0, b = 0;
        const uint32_t k = decode_tok<CL>(S, w0, p, nb, a, b);
        if (k == kErr) {
            stop = 2;
            break;
        }
        p += nb;
        if (k == kEob) {
            stop = 1;
            break;
        }
        cnt += k == kLit ? 1u : a;
        nmt += k == kMatch ? 1u : 0u;
    }
}

// DATA tokens through a per-lane 64-bit bit buffer over the staged words: a literal with a fast code costs one LDS
// lookup (the next stream word is read ahead every step); anything else (matches, long codes, end of block) goes
// through decode_tok at the buffer's position and re-seeks.
struct Dec {
    uint32_t p;      // stream bit of bb's bit 0
    uint64_t bb;     // stream bits [p, p + avail)
    uint32_t avail;  // > 32 after the refill at the top of a step
    uint32_t wi;     // stage index of wn
    uint32_t wn;     // stage[wi]
};

__device__ __forceinline__ void dec_seek(const Lds& S, uint32_t w0, Dec& d, uint32_t p) {
    const uint32_t i = (p >> 5) - w0, sh = p & 31u;
    const uint32_t x0 = S.stage[sw(i)], x1 = S.stage[sw(i + 1)];
    d.p = p;
    d.bb = (((uint64_t)x1 << 32) | x0) >> sh;
    d.avail = 64u - sh;
    d.wi = i + 2;
    d.wn = S.stage[sw(i + 2)];
}

__device__ __forceinline__ void dec_refill(const Lds& S, Dec& d) {
    const bool need = d.avail <= 32u;
    d.bb |= need ? ((uint64_t)d.wn << d.avail) : 0ull;
    d.avail += need ? 32u : 0u;
    d.wi += need ? 1u : 0u;
    d.wn = S.stage[sw(d.wi)];
}

__device__ __forceinline__ void dec_drop(Dec& d, uint32_t n) {
    d.bb >>= n;
    d.avail -= n;
    d.p += n;
}

// one token from the bit buffer.  Literal / length codes <= 15 bits + 5 extra fit the > 32 refilled bits; the buffer is
// refilled again before the distance code (<= 15 bits + 13 extra).
__device__ __forceinline__ uint32_t data_step(const Lds& S, Dec& d, uint32_t& a, uint32_t& b) {
    dec_refill(S, d);
    const uint32_t e = S.u.lit_fast[(uint32_t)d.bb & ((1u << kLitBits) - 1u)];
    if (e - 1u < (256u << 4) - 1u) {  // 0 < e < 256 << 4: a literal with a fast code
        a = e >> 4;
        dec_drop(d, e & 15u);
        return kLit;
    }
    uint32_t len, sym;
    if (e) {
        len = e & 15u;
        sym = e >> 4;
    } else if (!slow_code<kLitBits>(S.lit, (uint32_t)d.bb, len, sym)) {
        return kErr;
    }
    if (sym < 256) {
        a = sym;
        dec_drop(d, len);
        return kLit;
    }
    if (sym == 256) {
        dec_drop(d, len);
        return kEob;
    }
    const uint32_t li = sym - 257;
    if (li >= 29) return kErr;
    uint32_t le = 0, lb = li + 3;  // RFC 1951 3.2.5: 3..10 plain, then 4 per extra-bit count, 258
    if (li == 28) {
        lb = 258;
    } else if (li >= 8) {
        le = (li >> 2) - 1;
        lb = ((4u | (li & 3u)) << le) + 3;
    }
    a = lb + (((uint32_t)d.bb >> len) & ((1u << le) - 1u));
    dec_drop(d, len + le);
    dec_refill(S, d);
    const uint32_t lo = (uint32_t)d.bb;
    const uint32_t e2 = S.dist_fast[lo & ((1u << kDistBits) - 1u)];
    uint32_t dl, ds;
    if (e2) {
        dl = e2 & 15u;
        ds = e2 >> 4;
    } else if (!slow_code<kDistBits>(S.dist, lo, dl, ds)) {
        return kErr;
    }
    if (ds >= 30) return kErr;
    uint32_t de = 0, db = ds + 1;
    if (ds >= 4) {
        de = (ds >> 1) - 1;
        db = ((2u | (ds & 1u)) << de) + 1;
    }
    b = db + ((lo >> dl) & ((1u << de) - 1u));
    dec_drop(d, dl + de);
    return kMatch;
}

__device__ __forceinline__ void count_pass_data(const Lds& S, uint32_t w0, uint32_t& p, uint32_t to, uint32_t& cnt,
                                                uint32_t& nmt, uint32_t& stop) {
    cnt = 0;
    nmt = 0;
    stop = 0;
    Dec d;
    dec_seek(S, w0, d, p);
    while (d.p < to) {
        uint32_t a = 0, b = 0;
        const uint32_t k = data_step(S, d, a, b);
        if (k == kErr) {
            stop = 2;
            break;
        }
        if (k == kEob) {
            stop = 1;
            break;
        }
        cnt += k == kLit ? 1u : a;
        nmt += k == kMatch ? 1u : 0u;
    }
    p = d.p;
}

template <bool CL>
__device__ __forceinline__ void count_any(const Lds& S, uint32_t w0, uint32_t& p, uint32_t to, uint32_t& cnt,
                                         uint32_t& nmt, uint32_t& stop) {
    if (CL) count_pass<true>(S, w0, p, to, cnt, nmt, stop);
    else count_pass_data(S, w0, p, to, cnt, nmt, stop);
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

__device__ __forceinline__ uint32_t lens_slot(uint32_t k, uint32_t hlit) { return k < hlit ? k : 288 + (k - hlit); }

// One chunk of the lane-parallel decoder from the true token boundary P0 (see the file comment).
// DATA (CL false): output position op, the ring, matches against the window; `done` at the end-of-block token.
// CL: code lengths k = op of need in total into S.u.h.lens; `done` when all are read.
// Advances P0 / op, adapts seg; returns kPngOk or an error.
template <bool CL>
__device__ int run_chunk(Lds& S, const uint32_t* __restrict__ src, uint32_t nwords, uint32_t& P0, uint32_t& op,
                         uint32_t& seg, uint32_t need, uint32_t hlit, uint8_t* __restrict__ dst, uint32_t& flushed,
                         uint32_t out_len, bool& done) {
    const int lane = threadIdx.x & 63;
    done = false;
    if (P0 > nwords * 32u + 64u) return kPngErrShort;
    // stage the chunk's words
    const uint32_t w0 = P0 >> 5;
    const uint32_t nst = 2 * seg + 6;
    for (uint32_t i = lane; i < nst; i += 64) S.stage[sw(i)] = w0 + i < nwords ? src[w0 + i] : 0u;
    __builtin_amdgcn_wave_barrier();
    const uint32_t Sk = P0 + (uint32_t)lane * seg, Sn = Sk + seg;
    // lead-in: synchronise before the segment (lane 0 starts on the true boundary)
    uint32_t p = Sk >= P0 + kLead ? Sk - kLead : P0;
    if (lane == 0) p = P0;
    if (CL) {
        while (p < Sk) {
            uint32_t nb = 0, a = 0, b = 0;
            const uint32_t k = decode_tok<true>(S, w0, p, nb, a, b);
            p += k == kErr ? 1u : nb;
        }
    } else if (p < Sk) {
        Dec d;
        dec_seek(S, w0, d, p);
        while (d.p < Sk) {
            uint32_t a = 0, b = 0;
            if (data_step(S, d, a, b) == kErr) dec_seek(S, w0, d, d.p + 1);
        }
        p = d.p;
    }
    uint32_t start = p, cnt, nmt, stop;
    count_any<CL>(S, w0, p, Sn, cnt, nmt, stop);
    uint32_t E = p;
    const uint32_t cap = CL ? 0xFFFFFFFFu : kCap;
    int m = 0;
    uint32_t incl_c = 0, incl_m = 0;
    bool capped = false;
    for (int round = 0;; ++round) {
        incl_c = wave_incl_scan(cnt);
        incl_m = wave_incl_scan(nmt);
        uint64_t endm = __ballot(stop != 0);
        if (CL) endm |= __ballot(incl_c >= need);
        m = endm ? (int)__builtin_ctzll(endm) : 63;
        const uint64_t capm = __ballot(incl_c > cap || incl_m > (uint32_t)kMaxMatch);
        capped = false;
        if (capm) {
            const int mc = (int)__builtin_ctzll(capm) - 1;
            if (mc < m) {
                m = mc;
                capped = true;
            }
        }
        const uint32_t prevE = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)E, 0x138, 0xf, 0xf, false);  // wave_shr:1
        const bool bad = lane >= 1 && lane <= m && start != prevE;
        if (!__ballot(bad)) break;
        if (round >= 64) return kPngErrCode;  // cannot happen: every round fixes at least one more lane
        if (bad) {
            start = prevE;
            p = start;
            count_any<CL>(S, w0, p, Sn, cnt, nmt, stop);
            E = p;
        }
    }
    if (m < 0) {  // lane 0's segment alone overflows the ring: smaller segments (at kSegMin it cannot)
        seg = seg >= 4 * kSegMin ? seg >> 2 : kSegMin;
        return kPngOk;
    }
    const uint32_t stop_m = lane_of(stop, m);
    if (!CL && stop_m == 2) return kPngErrCode;
    if (CL && stop_m != 0 && lane_of(incl_c, m) < need) return kPngErrCode;
    if (!CL && op + lane_of(incl_c, m) > out_len) return kPngErrOverrun;
    // write pass: literals into place, matches listed in stream order
    uint32_t o = 0, mi = incl_m - nmt, werr = 0;
    const uint32_t o_end = op + need;  // CL only
    if (lane <= m) {
        o = op + (incl_c - cnt);
        p = start;
        if (CL) {
            while (p < Sn) {
                if (o >= o_end) break;
                uint32_t nb = 0, a = 0, b = 0;
                const uint32_t k = decode_tok<true>(S, w0, p, nb, a, b);
                if (k == kErr) break;
                p += nb;
                if (k == kLit) {
                    S.u.h.lens[lens_slot(o, hlit)] = (uint8_t)a;
                    ++o;
                } else if (k == kMatch) {
                    S.mdst[mi] = o;
                    S.mld[mi] = (a << 16) | b;
                    ++mi;
                    o += a;
                } else {
                    for (uint32_t j = 0; j < a; ++j)
                        if (o + j < o_end) S.u.h.lens[lens_slot(o + j, hlit)] = 0;
                    o += a;
                }
            }
            if (o > o_end) werr = 1;
        } else {
            Dec d;
            dec_seek(S, w0, d, p);
            while (d.p < Sn) {
                uint32_t a = 0, b = 0;
                const uint32_t k = data_step(S, d, a, b);
                if (k == kErr || k == kEob) break;
                if (k == kLit) {
                    S.ring[o & kRingMask] = (uint8_t)a;
                    ++o;
                } else {
                    S.mdst[mi] = o;
                    S.mld[mi] = (a << 16) | b;
                    ++mi;
                    o += a;
                }
            }
            p = d.p;
        }
    }
    if (__ballot(werr != 0)) return kPngErrCode;
    const uint32_t P1 = lane_of(p, m), op1 = lane_of(o, m), nm = lane_of(mi, m);
    __builtin_amdgcn_wave_barrier();
    // matches, in stream order
    const uint32_t ring_lo = op1 > (uint32_t)kRing ? op1 - kRing : 0u;  // older output is in HBM only
    bool fenced = false;
    for (uint32_t i = 0; i < nm; ++i) {
        const uint32_t d = uni(S.mdst[i]), ld = uni(S.mld[i]);
        const uint32_t L = ld >> 16, D = ld & 0xFFFFu;
        if (D > d) return kPngErrCode;
        if (CL) {
            const uint32_t v = S.u.h.lens[lens_slot(d - 1, hlit)];
            for (uint32_t j = lane; j < L; j += 64) S.u.h.lens[lens_slot(d + j, hlit)] = (uint8_t)v;
            __builtin_amdgcn_wave_barrier();
            continue;
        }
        const bool far = d - D < ring_lo;
        if (far && !fenced) {  // the output flushed so far must be visible to the loads below
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            fenced = true;
        }
        for (uint32_t j0 = 0; j0 < L; j0 += 64) {
            const uint32_t j = j0 + lane;
            uint32_t v = 0;
            if (j < L) {
                const uint32_t s = d - D + (D == 1 ? 0u : j % D);
                if (s >= ring_lo) {
                    v = S.ring[s & kRingMask];
                } else {
                    uint32_t* wp = reinterpret_cast<uint32_t*>(dst + (s & ~3u));
                    v = (__hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> (8 * (s & 3u))) & 0xFFu;
                }
            }
            __builtin_amdgcn_wave_barrier();
            if (j < L) S.ring[(d + j) & kRingMask] = (uint8_t)v;
            __builtin_amdgcn_wave_barrier();
        }
    }
    const uint32_t op0 = op;
    P0 = P1;
    if (CL) {
        op = op1;
        done = op1 >= o_end;
        return kPngOk;
    }
    // stream the completed 16-byte groups
    const uint32_t to = op1 & ~15u;
    __builtin_amdgcn_wave_barrier();
    flush(S, dst, flushed, to);
    flushed = to;
    __builtin_amdgcn_wave_barrier();
    op = op1;
    done = stop_m == 1;
    if (capped) seg = seg >= 2 * kSegMin ? seg >> 1 : kSegMin;
    else if (m == 63 && op1 - op0 < kCap / 4 && seg < kSegMax) seg <<= 1;
    return kPngOk;
}

// image i: zlib stream at src + off[i] (4-B aligned), len[i] bytes -> out_len bytes at out + i * out_pitch
__global__ __launch_bounds__(64) void inflate_kernel(const uint8_t* __restrict__ src, const int64_t* __restrict__ off,
                                                     const int32_t* __restrict__ len, uint8_t* __restrict__ out,
                                                     int64_t out_pitch, uint32_t out_len, int32_t* __restrict__ status,
                                                     int32_t* __restrict__ crc_bad, uint32_t* __restrict__ adler) {
    extern __shared__ __align__(16) uint8_t lds_raw[];
    Lds& S = *reinterpret_cast<Lds*>(lds_raw);
    const int img = blockIdx.x;
    const int lane = threadIdx.x & 63;
    uint8_t* dst = out + (int64_t)img * out_pitch;
    Bits br;
    br.src = reinterpret_cast<const uint32_t*>(src + off[img]);
    br.nwords = (uint32_t)(len[img] + 3) / 4;
    br.pos = 0;
    const uint32_t nbytes = (uint32_t)len[img];
    int32_t st = kPngOk;
    uint32_t op = 0, flushed = 0, seg = kSegMax;
    // an IDAT chunk whose CRC failed (gather_kernel, flag 1): libpng stops at it (a critical chunk's CRC error is
    // fatal); a file the host could not read or parse arrives flagged with its status (kPngErrFile) and no stream
    const int32_t flagged = (int32_t)uni((uint32_t)crc_bad[img]);
    if (flagged != 0) {
        if (lane == 0) {
            crc_bad[img] = 0;  // the flag is read (readfirstlane waited for it) before it is cleared for the slot's reuse
            status[img] = flagged == 1 ? kPngErrCrc : flagged;
        }
        return;
    }
    // zlib header (RFC 1950): CM 8, CINFO <= 7, no preset dictionary, FCHECK
    {
        const uint32_t cmf = br.get(8), flg = br.get(8);
        if ((cmf & 15u) != 8u || (cmf >> 4) > 7u || (flg & 32u) || ((cmf << 8) | flg) % 31u) st = kPngErrHeader;
    }
    bool last = false;
    while (st == kPngOk && !last) {
        if (br.pos > br.nwords * 32u) {
            st = kPngErrShort;
            break;
        }
        last = br.get(1) != 0;
        const uint32_t type = br.get(2);
        if (type == 0) {
            // stored block: byte-align, LEN, NLEN, LEN raw bytes (copied by the lanes through the ring)
            br.pos = (br.pos + 7u) & ~7u;
            const uint32_t n = br.get(16), nn = br.get(16);
            if ((n ^ 0xFFFFu) != nn) {
                st = kPngErrBlock;
                break;
            }
            if (op + n > out_len || (br.pos >> 3) + n > nbytes) {
                st = op + n > out_len ? kPngErrOverrun : kPngErrShort;
                break;
            }
            const uint8_t* sb = src + off[img] + (br.pos >> 3);
            for (uint32_t k0 = 0; k0 < n; k0 += 4096) {
                const uint32_t piece = min(4096u, n - k0);
                for (uint32_t k = lane; k < piece; k += 64) S.ring[(op + k) & kRingMask] = sb[k0 + k];
                op += piece;
                const uint32_t to = op & ~15u;
                __builtin_amdgcn_wave_barrier();
                flush(S, dst, flushed, to);
                flushed = to;
                __builtin_amdgcn_wave_barrier();
            }
            br.pos += 8u * n;
            continue;
        }
        if (type == 3) {
            st = kPngErrBlock;
            break;
        }
        if (type == 1) {
            // fixed codes (RFC 1951 3.2.6)
            for (int s = lane; s < 320; s += 64) S.u.h.lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : 5;
            __builtin_amdgcn_wave_barrier();
        } else {
            const uint32_t hlit = br.get(5) + 257, hdist = br.get(5) + 1, hclen = br.get(4) + 4;
            if (hlit > 286 || hdist > 30) {
                st = kPngErrBlock;
                break;
            }
            if (lane < 20) S.u.h.cl[lane] = 0;
            __builtin_amdgcn_wave_barrier();
            {
                // hclen 3-bit lengths in the order 16 17 18 0 8 7 9 6 10 5 11 4 12 3 13 2 14 1 15: lane k takes the k-th
                const uint32_t pos0 = br.pos;
                if ((uint32_t)lane < hclen) {
                    const uint32_t q = pos0 + 3u * lane, w = q >> 5, sh = q & 31u;
                    const uint64_t x = (((uint64_t)br.word(w + 1) << 32) | br.word(w)) >> sh;
                    S.u.h.cl[kClOrder[lane]] = (uint8_t)(x & 7u);
                }
                br.pos = pos0 + 3u * hclen;
            }
            __builtin_amdgcn_wave_barrier();
            // the code-length code: its table in dist_fast / dist (7-bit codes)
            if (!build_table(S.u.h.cl, 19, S.dist, S.dist_fast, kClBits)) {
                st = kPngErrCode;
                break;
            }
            // hlit + hdist code lengths, litlen into lens[0, hlit), distance into lens[288, 288 + hdist)
            for (int s = lane; s < 320; s += 64) S.u.h.lens[s] = 0;
            __builtin_amdgcn_wave_barrier();
            uint32_t k = 0, P = br.pos, cseg = kSegMin;
            const uint32_t total = hlit + hdist;
            bool done = false;
            while (!done) {
                st = run_chunk<true>(S, br.src, br.nwords, P, k, cseg, total - k, hlit, dst, flushed, out_len, done);
                if (st != kPngOk) break;
            }
            if (st != kPngOk) break;
            br.pos = P;
            __builtin_amdgcn_wave_barrier();
            if (uni(S.u.h.lens[256]) == 0) {  // no end-of-block code
                st = kPngErrCode;
                break;
            }
        }
        if (!build_table(S.u.h.lens + 288, 30, S.dist, S.dist_fast, kDistBits) ||
            !build_table(S.u.h.lens, 288, S.lit, S.u.lit_fast, kLitBits)) {  // last: lit_fast overlays lens
            st = kPngErrCode;
            break;
        }
        // the block's tokens
        uint32_t P = br.pos;
        bool done = false;
        while (!done) {
            st = run_chunk<false>(S, br.src, br.nwords, P, op, seg, 0xFFFFFFFFu, 0, dst, flushed, out_len, done);
            if (st != kPngOk) break;
        }
        if (st != kPngOk) break;
        br.pos = P;
    }
    if (st == kPngOk && br.pos > br.nwords * 32u) st = kPngErrShort;  // decoding ran past the stream
    if (st == kPngOk && op != out_len) st = kPngErrShort;
    // the zlib trailer: Adler-32 of the inflated bytes, big-endian, at the next byte boundary (RFC 1950 2.2)
    if (st == kPngOk && adler) {  // (null: the Adler-32 check is off, yv_pngdec_set_checks)
        br.pos = (br.pos + 7u) & ~7u;
        if ((br.pos >> 3) + 4u > nbytes) {
            st = kPngErrAdler;  // no trailer: zlib never reports the stream's end
        } else {
            const uint32_t b0 = br.get(8), b1 = br.get(8), b2 = br.get(8), b3 = br.get(8);
            if (lane == 0) adler[img] = (b0 << 24) | (b1 << 16) | (b2 << 8) | b3;
        }
    }
    __builtin_amdgcn_wave_barrier();
    if (st == kPngOk) flush(S, dst, flushed, op);
    if (lane == 0) status[img] = st;
}

__device__ __forceinline__ uint32_t byte_of(uint32_t v, int k) { return (v >> (8 * k)) & 0xFFu; }

// Adler-32 sums of the inflated stream, per lane: s1 = sum d_i, s2 = sum i d_i over the bytes the lane read (i = the
// byte's position in the stream).  A dword x of nb valid bytes at position pos: v_dot4 gives sum d and sum k d_k.
struct AdlerAcc {
    uint64_t s1 = 0, s2 = 0;
    __device__ __forceinline__ void add_dword(uint32_t x, int nb, uint64_t pos) {
        if (nb < 4) x &= nb <= 0 ? 0u : (0xFFFFFFFFu >> (8 * (4 - nb)));
        const uint32_t t = __builtin_amdgcn_udot4(x, 0x01010101u, 0u, false);
        const uint32_t u = __builtin_amdgcn_udot4(x, 0x03020100u, 0u, false);
        s1 += t;
        s2 += pos * t + u;
    }
    __device__ __forceinline__ void add_byte(uint32_t d, uint64_t pos) {
        s1 += d;
        s2 += pos * d;
    }
};

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// adler32 of n bytes from the sums: a = 1 + s1, b = n + sum (n - i) d_i = n + n s1 - s2 (mod 65521)
__device__ __forceinline__ uint32_t adler_of(uint64_t s1, uint64_t s2, uint64_t n) {
    const uint64_t a = (1u + s1) % 65521u;
    const uint64_t b = (n + n * s1 - s2) % 65521u;
    return (uint32_t)((b << 16) | a);
}

// Any filter types: a wavefront over rows (see the file comment), one 4-byte group per lane per step.
// returns true (wave-uniform) when a row has a filter type > 4
__device__ bool unfilter_wavefront(const uint8_t* __restrict__ rimg, int H, int W, uint8_t* __restrict__ dimg,
                                   int dst_stride, AdlerAcc& acc) {
    const int lane = threadIdx.x & 63;
    const int G = (W + 3) >> 2;  // 4-byte groups per row
    int bad = 0;
    for (int r0 = 0; r0 < H; r0 += 64) {
        const int r = r0 + lane;
        const bool row_ok = r < H;
        const uint8_t* rr = rimg + (int64_t)(row_ok ? r : 0) * (W + 1);
        const int f = row_ok ? rr[0] : 0;
        bad |= f > 4 ? 1 : 0;
        if (row_ok) acc.add_byte((uint32_t)f, (uint64_t)r * (W + 1));
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
                acc.add_dword(x, nb, (uint64_t)r * (W + 1) + 1 + 4 * g);
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
    return __ballot(bad != 0) != 0;
}


// bytewise a + b mod 256 in each of the four bytes
__device__ __forceinline__ uint32_t add8(uint32_t a, uint32_t b) {
    return ((a & 0x7F7F7F7Fu) + (b & 0x7F7F7F7Fu)) ^ ((a ^ b) & 0x80808080u);
}

// Rows filtered None / Sub / Up only (cv::imwrite writes Sub rows): no dependency between bytes beyond a running sum, so
// the 64 lanes share each row, lane l owning its bytes [4 NW l, 4 NW (l + 1)).  Sub = a prefix sum mod 256 along the
// row: within the lane's dwords by shifted bytewise adds, across lanes by a wave scan of the lanes' sums.  Up adds the
// row above, which the same lane made one row earlier.  Rows stream through registers PF rows ahead of their use.
template <int NW>
__device__ void unfilter_rowwise(const uint8_t* __restrict__ rimg, int H, int W, uint8_t* __restrict__ dimg,
                                 int dst_stride, AdlerAcc& acc) {
    constexpr int PF = 4;
    const int lane = threadIdx.x & 63;
    const int b0 = 4 * NW * lane;
    const int nb = min(max(W - b0, 0), 4 * NW);
    uint32_t buf[PF][NW], fb[PF], prev[NW];
#pragma unroll
    for (int i = 0; i < NW; ++i) prev[i] = 0;
    auto load = [&](int r, uint32_t* x, uint32_t& f) {
        if (r < H) {
            const uint8_t* rr = rimg + (int64_t)r * (W + 1);
            f = rr[0];
            if (nb > 0) __builtin_memcpy(x, rr + 1 + b0, 4 * NW);  // the last lane may over-read: the buffer is padded
        }
    };
#pragma unroll
    for (int k = 0; k < PF; ++k) load(k, buf[k], fb[k]);
    for (int r0 = 0; r0 < H; r0 += PF) {
#pragma unroll
        for (int k = 0; k < PF; ++k) {
            const int r = r0 + k;
            if (r >= H) break;
            uint32_t x[NW];
#pragma unroll
            for (int i = 0; i < NW; ++i) x[i] = buf[k][i];
            const uint32_t f = uni(fb[k]);
            load(r + PF, buf[k], fb[k]);
            {  // the row's raw bytes into the Adler sums: this lane's dwords, the filter byte on lane 0
                const uint64_t rpos = (uint64_t)r * (W + 1);
                uint32_t T = 0, Q = 0;
#pragma unroll
                for (int i = 0; i < NW; ++i) {
                    const int vb = nb - 4 * i;
                    uint32_t xi = x[i];
                    if (vb < 4) xi &= vb <= 0 ? 0u : (0xFFFFFFFFu >> (8 * (4 - vb)));
                    const uint32_t t = __builtin_amdgcn_udot4(xi, 0x01010101u, 0u, false);
                    T += t;
                    Q += (uint32_t)(4 * i) * t + __builtin_amdgcn_udot4(xi, 0x03020100u, 0u, false);
                }
                acc.s1 += T;
                acc.s2 += (rpos + 1 + b0) * T + Q;
                if (lane == 0) acc.add_byte(f, rpos);
            }
            if (f == 1) {
                uint32_t carry = 0;
#pragma unroll
                for (int i = 0; i < NW; ++i) {
                    uint32_t y = add8(x[i], x[i] << 8);
                    y = add8(y, y << 16);
                    y = add8(y, carry * 0x01010101u);
                    carry = y >> 24;
                    x[i] = y;
                }
                const uint32_t c = (wave_incl_scan(carry) - carry) & 0xFFu;
#pragma unroll
                for (int i = 0; i < NW; ++i) x[i] = add8(x[i], c * 0x01010101u);
            } else if (f == 2) {
#pragma unroll
                for (int i = 0; i < NW; ++i) x[i] = add8(x[i], prev[i]);
            }
#pragma unroll
            for (int i = 0; i < NW; ++i) prev[i] = x[i];
            uint8_t* po = dimg + (int64_t)r * dst_stride + b0;
            if (nb == 4 * NW) {
                __builtin_memcpy(po, x, 4 * NW);
            } else {
#pragma unroll
                for (int i = 0; i < NW; ++i)
#pragma unroll
                    for (int k2 = 0; k2 < 4; ++k2)
                        if (4 * i + k2 < nb) po[4 * i + k2] = (uint8_t)(x[i] >> (8 * k2));
            }
        }
    }
}

// PNG scanline filters (filter method 0) of 8-bit grey rows: raw rows of 1 + W bytes (filter type first) -> rows of W
// bytes at dst + i * dst_pitch with row stride dst_stride.  NW = ceil(W / 256) (0: W > 4096): images whose rows are all
// None / Sub / Up take the row-wise path, others the wavefront.
// a failed image: zeros (cv::imread's empty Mat has no pixels; the caller sees the status)
__device__ void zero_image(uint8_t* __restrict__ dimg, int H, int W, int dst_stride) {
    const int lane = threadIdx.x & 63;
    for (int r = 0; r < H; ++r)
        for (int c = lane; c < W; c += 64) dimg[(int64_t)r * dst_stride + c] = 0;
}

// the image's status after its filters (wave-uniform): kPngOk or kPngErrFilter
template <int NW>
__device__ int32_t unfilter_body(const uint8_t* __restrict__ rimg, int H, int W, uint8_t* __restrict__ dimg,
                                 int dst_stride, AdlerAcc& acc) {
    const int lane = threadIdx.x & 63;
    if (NW > 0) {
        bool rowwise = true, bad = false;
        for (int r = lane; r < H; r += 64) {
            const uint32_t f = rimg[(int64_t)r * (W + 1)];
            rowwise = rowwise && f <= 2;
            bad = bad || f > 4;
        }
        if (__ballot(bad)) return kPngErrFilter;
        if (!__ballot(!rowwise)) {
            unfilter_rowwise<(NW > 0 ? NW : 1)>(rimg, H, W, dimg, dst_stride, acc);
            return kPngOk;
        }
    }
    return unfilter_wavefront(rimg, H, W, dimg, dst_stride, acc) ? kPngErrFilter : kPngOk;
}

template <int NW>
__global__ __launch_bounds__(64) void unfilter_kernel(const uint8_t* __restrict__ raw, int64_t raw_pitch, int H, int W,
                                                      uint8_t* __restrict__ dst, int64_t dst_pitch, int dst_stride,
                                                      int32_t* __restrict__ status, const uint32_t* __restrict__ adler,
                                                      uint32_t* __restrict__ bad_total) {
    const int img = blockIdx.x;
    const int lane = threadIdx.x & 63;
    const uint8_t* rimg = raw + (int64_t)img * raw_pitch;
    uint8_t* dimg = dst + (int64_t)img * dst_pitch;
    int32_t st = (int32_t)uni((uint32_t)status[img]);
    if (st == kPngOk) {
        AdlerAcc acc;
        st = unfilter_body<NW>(rimg, H, W, dimg, dst_stride, acc);
        if (st == kPngOk && adler) {
            const uint64_t s1 = wave_sum_u64(acc.s1), s2 = wave_sum_u64(acc.s2);
            if (adler_of(s1, s2, (uint64_t)H * (W + 1)) != uni(adler[img])) st = kPngErrAdler;
        }
        if (st != kPngOk && lane == 0) status[img] = st;
    }
    if (st != kPngOk) {
        zero_image(dimg, H, W, dst_stride);
        if (lane == 0) atomicAdd(bad_total, 1u);
    }
}
// IDAT payloads of the staged files -> contiguous zlib streams: one wave per payload, 16 bytes per lane per pass; then
// the chunk's CRC-32 over its type and data (each lane one contiguous segment, slice-by-8 from LDS tables, the 64
// segment CRCs joined pairwise up a tree), against the stored big-endian CRC after the data
__global__ __launch_bounds__(64) void gather_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                   const PngPiece* __restrict__ pieces, int32_t* __restrict__ crc_bad) {
    __shared__ uint32_t s_tab[8][256];
    const int lane = threadIdx.x & 63;
    if (crc_bad)
        for (int i = lane; i < 8 * 256; i += 64) s_tab[i >> 8][i & 255] = kCrcTab.t[i >> 8][i & 255];
    const PngPiece pc = pieces[blockIdx.x];
    const uint8_t* s = src + pc.src;
    uint8_t* d = dst + pc.dst;
    for (int64_t i = 16 * lane; i < pc.len; i += 1024) {
        if (i + 16 <= pc.len) {
            uint4 v;
            __builtin_memcpy(&v, s + i, 16);
            __builtin_memcpy(d + i, &v, 16);
        } else {
            for (int64_t k = i; k < pc.len; ++k) d[k] = s[k];
        }
    }
    if (!crc_bad) return;  // checks off (yv_pngdec_set_checks)
    __syncthreads();  // the tables
    const uint8_t* c0 = s - 4;  // chunk type, then the data
    const uint32_t total = (uint32_t)pc.len + 4u;
    const uint32_t seg = (((total + 63u) / 64u) + 7u) & ~7u;
    const uint32_t lo = min((uint32_t)lane * seg, total), hi = min(lo + seg, total);
    uint32_t c = 0xFFFFFFFFu;
    uint32_t p = lo;
    for (; p + 8u <= hi; p += 8u) {
        uint32_t w0, w1;
        __builtin_memcpy(&w0, c0 + p, 4);
        __builtin_memcpy(&w1, c0 + p + 4, 4);
        w0 ^= c;
        c = s_tab[7][w0 & 255u] ^ s_tab[6][(w0 >> 8) & 255u] ^ s_tab[5][(w0 >> 16) & 255u] ^ s_tab[4][w0 >> 24] ^
            s_tab[3][w1 & 255u] ^ s_tab[2][(w1 >> 8) & 255u] ^ s_tab[1][(w1 >> 16) & 255u] ^ s_tab[0][w1 >> 24];
    }
    for (; p < hi; ++p) c = s_tab[0][(c ^ c0[p]) & 255u] ^ (c >> 8);
    c ^= 0xFFFFFFFFu;
    uint32_t n = hi - lo;
    // lanes l and l + off (off = 1, 2, 4, ...): lane l's span is followed by lane l + off's
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t cb = (uint32_t)__shfl_down((int)c, off, 64), nb = (uint32_t)__shfl_down((int)n, off, 64);
        if ((lane & (2 * off - 1)) == 0) {
            c = crc_combine(c, cb, nb);
            n += nb;
        }
    }
    if (lane == 0) {
        const uint8_t* t = s + pc.len;
        const uint32_t stored = ((uint32_t)t[0] << 24) | ((uint32_t)t[1] << 16) | ((uint32_t)t[2] << 8) | t[3];
        if (stored != c) crc_bad[pc.img] = 1;
    }
}

}  // namespace png

void launch_png_gather(const uint8_t* src, uint8_t* dst, const PngPiece* pieces, int n, int32_t* crc_bad,
                       hipStream_t s) {
    if (n > 0) hipLaunchKernelGGL(png::gather_kernel, dim3(n), dim3(64), 0, s, src, dst, pieces, crc_bad);
}

void launch_png_inflate(const uint8_t* src, const int64_t* off, const int32_t* len, int n, uint8_t* out,
                        int64_t out_pitch, uint32_t out_len, int32_t* status, int32_t* crc_bad, uint32_t* adler,
                        hipStream_t s) {
    hipLaunchKernelGGL(png::inflate_kernel, dim3(n), dim3(64), sizeof(png::Lds), s, src, off, len, out, out_pitch,
                       out_len, status, crc_bad, adler);
}

void launch_png_unfilter(const uint8_t* raw, int64_t raw_pitch, int n, int H, int W, uint8_t* dst, int64_t dst_pitch,
                         int dst_stride, int32_t* status, const uint32_t* adler, uint32_t* bad_total, hipStream_t s) {
    const int nw = (W + 255) / 256;
#define YV_UNFILTER(NW)                                                                                              \
    hipLaunchKernelGGL(png::unfilter_kernel<NW>, dim3(n), dim3(64), 0, s, raw, raw_pitch, H, W, dst, dst_pitch,     \
                       dst_stride, status, adler, bad_total)
    switch (nw) {
    case 1: YV_UNFILTER(1); break;
    case 2: YV_UNFILTER(2); break;
    case 3: YV_UNFILTER(3); break;
    case 4: YV_UNFILTER(4); break;
    case 5: YV_UNFILTER(5); break;
    case 6: YV_UNFILTER(6); break;
    case 7: YV_UNFILTER(7); break;
    case 8: YV_UNFILTER(8); break;
    case 9: case 10: YV_UNFILTER(10); break;
    case 11: case 12: YV_UNFILTER(12); break;
    case 13: case 14: case 15: case 16: YV_UNFILTER(16); break;
    default: YV_UNFILTER(0); break;
    }
#undef YV_UNFILTER
}

}  // namespace yavo
