// yavo_io.hip -- host side of frame I/O (include/yavo/yavo_io.h): PNG -> 8-bit grey on zlib,
// the sorted KITTI image listing, calib.txt, the KITTI pose format, and a threaded decoder feeding pinned staging
// whose copies to HBM run asynchronously on the caller's stream.  Host code only (no kernels).
#include <hip/hip_runtime.h>
#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/yavo/yavo_io.h"
#include "yavo_internal.h"

namespace {

uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

struct PngHeader {
    int W = 0, H = 0, depth = 0, ctype = 0, interlace = 0;
};

// chunk walk: IHDR, PLTE, the concatenated IDAT stream; stops at IEND
int png_parse(const uint8_t* d, size_t len, PngHeader& h, std::vector<uint8_t>* idat, std::vector<uint8_t>* plte) {
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (!d || len < 8 + 25 || std::memcmp(d, sig, 8) != 0) return YV_ERR_INVALID;
    size_t off = 8;
    bool have_ihdr = false;
    while (off + 12 <= len) {
        const uint32_t n = be32(d + off);
        const uint8_t* type = d + off + 4;
        const uint8_t* body = d + off + 8;
        if (n > len - off - 12) return YV_ERR_INVALID;
        if (!std::memcmp(type, "IHDR", 4)) {
            if (n != 13) return YV_ERR_INVALID;
            h.W = (int)be32(body);
            h.H = (int)be32(body + 4);
            h.depth = body[8];
            h.ctype = body[9];
            if (body[10] != 0 || body[11] != 0) return YV_ERR_INVALID;  // compression / filter method
            h.interlace = body[12];
            have_ihdr = true;
            if (!idat && !plte) return YV_OK;
        } else if (!std::memcmp(type, "PLTE", 4)) {
            if (plte) plte->assign(body, body + n);
        } else if (!std::memcmp(type, "IDAT", 4)) {
            if (idat) idat->insert(idat->end(), body, body + n);
        } else if (!std::memcmp(type, "IEND", 4)) {
            break;
        }
        off += 12 + n;
    }
    return have_ihdr ? YV_OK : YV_ERR_INVALID;
}

int png_channels(int ctype) {
    switch (ctype) {
        case 0: return 1;
        case 2: return 3;
        case 3: return 1;
        case 4: return 2;
        case 6: return 4;
        default: return 0;
    }
}

bool png_supported(const PngHeader& h) {
    if (h.W <= 0 || h.H <= 0 || (int64_t)h.W * h.H > (1ll << 30) || h.interlace != 0) return false;
    switch (h.ctype) {
        case 0: return h.depth == 1 || h.depth == 2 || h.depth == 4 || h.depth == 8 || h.depth == 16;
        case 3: return h.depth == 1 || h.depth == 2 || h.depth == 4 || h.depth == 8;
        case 4: return h.depth == 8 || h.depth == 16;
        case 2:
        case 6: return h.depth == 8;
        default: return false;
    }
}

// libpng png_do_rgb_to_gray, 8-bit, no gamma table: coefficients (29900, 58700) / 100000 * 32768 truncated
inline uint8_t rgb_to_gray(uint32_t r, uint32_t g, uint32_t b) {
    constexpr uint32_t rc = 9797, gc = 19234, bc = 32768 - rc - gc;
    if (r == g && r == b) return (uint8_t)r;
    return (uint8_t)((rc * r + gc * g + bc * b) >> 15);
}

uint8_t paeth(int a, int b, int c) {
    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    if (pa <= pb && pa <= pc) return (uint8_t)a;
    if (pb <= pc) return (uint8_t)b;
    return (uint8_t)c;
}

int png_decode(const uint8_t* data, size_t len, uint8_t* dst, int stride, int H, int W) {
    PngHeader h;
    std::vector<uint8_t> idat, plte;
    if (png_parse(data, len, h, &idat, &plte) != YV_OK) return YV_ERR_INVALID;
    if (!png_supported(h) || h.H != H || h.W != W || stride < W) return YV_ERR_INVALID;
    const int ch = png_channels(h.ctype);
    const size_t bits = (size_t)ch * h.depth;
    const size_t rowb = ((size_t)W * bits + 7) / 8;
    const size_t fbpp = std::max<size_t>(1, bits / 8);
    std::vector<uint8_t> raw((rowb + 1) * (size_t)H);
    z_stream zs;
    std::memset(&zs, 0, sizeof zs);
    if (inflateInit(&zs) != Z_OK) return YV_ERR_INVALID;
    zs.next_in = idat.data();
    zs.avail_in = (uInt)idat.size();
    zs.next_out = raw.data();
    zs.avail_out = (uInt)raw.size();
    const int zr = inflate(&zs, Z_FINISH);
    const size_t produced = raw.size() - zs.avail_out;
    inflateEnd(&zs);
    if ((zr != Z_STREAM_END && zr != Z_BUF_ERROR && zr != Z_OK) || produced != raw.size()) return YV_ERR_INVALID;
    // unfilter in place: row y = raw[y (rowb + 1) + 1 ..], filter byte first
    for (int y = 0; y < H; ++y) {
        uint8_t* row = raw.data() + (size_t)y * (rowb + 1);
        const uint8_t f = row[0];
        uint8_t* cur = row + 1;
        const uint8_t* prev = y ? raw.data() + (size_t)(y - 1) * (rowb + 1) + 1 : nullptr;
        switch (f) {
            case 0: break;
            case 1:
                for (size_t i = fbpp; i < rowb; ++i) cur[i] = (uint8_t)(cur[i] + cur[i - fbpp]);
                break;
            case 2:
                if (prev)
                    for (size_t i = 0; i < rowb; ++i) cur[i] = (uint8_t)(cur[i] + prev[i]);
                break;
            case 3:
                for (size_t i = 0; i < rowb; ++i) {
                    const int a = i >= fbpp ? cur[i - fbpp] : 0, b = prev ? prev[i] : 0;
                    cur[i] = (uint8_t)(cur[i] + ((a + b) >> 1));
                }
                break;
            case 4:
                if (fbpp == 1 && prev) {
                    // 8-bit grey rows below the first: a (left) and c (upper left) carried in registers and the
                    // predictor picked without branches, p - a = b - c, p - b = a - c, p - c = a + b - 2c
                    int a = 0, c = 0;
                    for (size_t i = 0; i < rowb; ++i) {
                        const int b = prev[i];
                        const int pa = std::abs(b - c), pb = std::abs(a - c), pc = std::abs(a + b - 2 * c);
                        const int pred = (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
                        a = (uint8_t)(cur[i] + pred);
                        cur[i] = (uint8_t)a;
                        c = b;
                    }
                    break;
                }
                for (size_t i = 0; i < rowb; ++i) {
                    const int a = i >= fbpp ? cur[i - fbpp] : 0, b = prev ? prev[i] : 0;
                    const int c = (prev && i >= fbpp) ? prev[i - fbpp] : 0;
                    cur[i] = (uint8_t)(cur[i] + paeth(a, b, c));
                }
                break;
            default: return YV_ERR_INVALID;
        }
    }
    for (int y = 0; y < H; ++y) {
        const uint8_t* s = raw.data() + (size_t)y * (rowb + 1) + 1;
        uint8_t* o = dst + (size_t)y * stride;
        if (h.ctype == 0 && h.depth == 8) {
            std::memcpy(o, s, (size_t)W);
        } else if (h.ctype == 0 && h.depth == 16) {
            for (int x = 0; x < W; ++x) o[x] = s[2 * x];  // png_set_strip_16: the high byte
        } else if (h.ctype == 0 || h.ctype == 3) {
            const int d = h.depth, per = 8 / std::min(d, 8);
            for (int x = 0; x < W; ++x) {
                uint32_t v;
                if (d == 8) {
                    v = s[x];
                } else {
                    const int byte = x / per, shift = 8 - d * (x % per + 1);
                    v = (s[byte] >> shift) & ((1u << d) - 1);
                }
                if (h.ctype == 0) {
                    o[x] = (uint8_t)(d == 8 ? v : v * 255 / ((1u << d) - 1));  // expand_gray_1_2_4_to_8
                } else {
                    if (3 * v + 2 >= plte.size()) return YV_ERR_INVALID;
                    o[x] = rgb_to_gray(plte[3 * v], plte[3 * v + 1], plte[3 * v + 2]);
                }
            }
        } else if (h.ctype == 4) {
            const int step = h.depth == 16 ? 4 : 2;
            for (int x = 0; x < W; ++x) o[x] = s[step * x];  // grey (high byte), alpha dropped
        } else {  // 2 / 6, 8-bit
            for (int x = 0; x < W; ++x) {
                const uint8_t* p = s + (size_t)ch * x;
                o[x] = rgb_to_gray(p[0], p[1], p[2]);
            }
        }
    }
    return YV_OK;
}

bool read_file(const std::string& path, std::vector<uint8_t>& out) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    out.clear();
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) out.insert(out.end(), buf, buf + n);
    const bool ok = !std::ferror(f);
    std::fclose(f);
    return ok;
}

// getFilesInFolder: every entry of the directory ('.' and '..' excluded), sorted as paths of one directory compare
bool list_sorted(const std::string& dir, std::vector<std::string>& out) {
    DIR* d = opendir(dir.c_str());
    if (!d) return false;
    std::vector<std::string> names;
    while (dirent* e = readdir(d)) {
        if (!std::strcmp(e->d_name, ".") || !std::strcmp(e->d_name, "..")) continue;
        names.emplace_back(e->d_name);
    }
    closedir(d);
    std::sort(names.begin(), names.end());
    std::string base = dir;
    if (!base.empty() && base.back() != '/') base += '/';
    out.clear();
    for (auto& n : names) out.push_back(base + n);
    return true;
}

// parseCalibString: split on ' ', std::stod each token (leading blanks allowed, trailing text ignored), skip failures
int parse_calib(const char* line, double out[16]) {
    std::vector<double> v;
    const std::string s(line ? line : "");
    size_t pos = 0;
    while (pos <= s.size()) {
        size_t next = s.find(' ', pos);
        if (next == std::string::npos) next = s.size();
        const std::string tok = s.substr(pos, next - pos);
        if (!tok.empty()) {
            const char* c = tok.c_str();
            char* end = nullptr;
            errno = 0;
            const double d = std::strtod(c, &end);
            if (end != c && errno != ERANGE) v.push_back(d);
        }
        pos = next + 1;
        if (next == s.size()) break;
    }
    for (int i = 0; i < 16; ++i) out[i] = i < (int)v.size() ? v[i] : 0.0;
    return (int)v.size();
}

// Eigen::Quaterniond::toRotationMatrix
void quat_to_R(const double* q, double* R) {
    const double x = q[0], y = q[1], z = q[2], w = q[3];
    const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz; R[2] = txz + twy;
    R[3] = txy + twz; R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy; R[7] = tyz + twx; R[8] = 1 - (txx + tyy);
}

}  // namespace

struct yv_seq {
    std::string dir;
    bool stereo = false;
    std::vector<std::string> left, right;
    int H = 0, W = 0;
    // pinned staging for yv_seq_upload: two slots, each reused after its copy completed
    uint8_t* stage[2] = {nullptr, nullptr};
    size_t stage_cap[2] = {0, 0};
    hipEvent_t done[2] = {nullptr, nullptr};
    bool pending[2] = {false, false};
    int next = 0;
};

namespace {

int decode_frames(yv_seq* s, int first, int n, uint8_t* dst, int64_t pitch, int threads) {
    const int per = s->stereo ? 2 : 1;
    const int total = n * per;
    if (threads <= 0) threads = (int)std::min<unsigned>(std::max(1u, std::thread::hardware_concurrency()), 64u);
    threads = std::max(1, std::min(threads, total));
    std::atomic<int> next{0}, status{YV_OK};
    auto work = [&]() {
        std::vector<uint8_t> file;
        for (int k; (k = next.fetch_add(1)) < total;) {
            const int frame = first + k / per, side = k % per;
            const std::string& path = side ? s->right[frame] : s->left[frame];
            if (!read_file(path, file)) {
                status = YV_ERR_INVALID;
                continue;
            }
            if (png_decode(file.data(), file.size(), dst + (int64_t)k * pitch, s->W, s->H, s->W) != YV_OK)
                status = YV_ERR_INVALID;
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; ++t) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
    return status.load();
}

}  // namespace

extern "C" {

int yv_png_info(const uint8_t* data, size_t len, int* H, int* W) {
    if (!H || !W) return YV_ERR_INVALID;
    PngHeader h;
    if (png_parse(data, len, h, nullptr, nullptr) != YV_OK || !png_supported(h)) return YV_ERR_INVALID;
    *H = h.H;
    *W = h.W;
    return YV_OK;
}

int yv_png_decode_gray(const uint8_t* data, size_t len, uint8_t* dst, int stride, int H, int W) {
    if (!data || !dst) return YV_ERR_INVALID;
    return png_decode(data, len, dst, stride, H, W);
}

int yv_imread_gray(const char* path, uint8_t* dst, int stride, int cap_h, int cap_w, int* H, int* W) {
    if (!path || !dst || !H || !W) return YV_ERR_INVALID;
    std::vector<uint8_t> file;
    if (!read_file(path, file)) return YV_ERR_INVALID;
    int h = 0, w = 0;
    if (yv_png_info(file.data(), file.size(), &h, &w) != YV_OK) return YV_ERR_INVALID;
    *H = h;
    *W = w;
    if (h > cap_h || w > cap_w || stride < w) return YV_ERR_CAPACITY;
    return png_decode(file.data(), file.size(), dst, stride, h, w);
}

int yv_parse_calib_string(const char* line, double out[16]) {
    if (!line || !out) return YV_ERR_INVALID;
    return parse_calib(line, out);
}

int yv_seq_open(const char* sequence_dir, int stereo, yv_seq** out) {
    if (!sequence_dir || !out) return YV_ERR_INVALID;
    *out = nullptr;
    yv_seq* s = new (std::nothrow) yv_seq();
    if (!s) return YV_ERR_INVALID;
    s->dir = sequence_dir;
    if (!s->dir.empty() && s->dir.back() != '/') s->dir += '/';
    s->stereo = stereo != 0;
    if (!list_sorted(s->dir + "image_0/", s->left) || s->left.empty() ||
        (s->stereo && (!list_sorted(s->dir + "image_1/", s->right) || s->right.size() < s->left.size()))) {
        delete s;
        return YV_ERR_INVALID;
    }
    std::vector<uint8_t> file;
    if (!read_file(s->left[0], file) || yv_png_info(file.data(), file.size(), &s->H, &s->W) != YV_OK) {
        delete s;
        return YV_ERR_INVALID;
    }
    *out = s;
    return YV_OK;
}

void yv_seq_close(yv_seq* s) {
    if (!s) return;
    for (int k = 0; k < 2; ++k) {
        if (s->done[k]) {
            (void)hipEventSynchronize(s->done[k]);
            (void)hipEventDestroy(s->done[k]);
        }
        if (s->stage[k]) (void)hipHostFree(s->stage[k]);
    }
    delete s;
}

int yv_seq_frames(const yv_seq* s) { return s ? (int)s->left.size() : YV_ERR_INVALID; }

int yv_seq_path(const yv_seq* s, int frame, int side, char* buf, int cap) {
    if (!s || !buf || frame < 0 || frame >= (int)s->left.size() || side < 0 || side > (s->stereo ? 1 : 0))
        return YV_ERR_INVALID;
    const std::string& p = side ? s->right[frame] : s->left[frame];
    if ((int)p.size() + 1 > cap) return YV_ERR_CAPACITY;
    std::memcpy(buf, p.c_str(), p.size() + 1);
    return (int)p.size();
}

int yv_seq_calib(const yv_seq* s, double P0[16], double P1[16], double K0[9], double K1[9]) {
    if (!s) return YV_ERR_INVALID;
    FILE* f = std::fopen((s->dir + "calib.txt").c_str(), "r");
    if (!f) return YV_ERR_INVALID;
    double P[2][16];
    for (int i = 0; i < 2; ++i) {
        std::string line;
        int c;
        while ((c = std::fgetc(f)) != EOF && c != '\n') line.push_back((char)c);
        parse_calib(line.c_str(), P[i]);
    }
    std::fclose(f);
    for (int i = 0; i < 16; ++i) {
        if (P0) P0[i] = P[0][i];
        if (P1) P1[i] = P[1][i];
    }
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {  // Camera::K = fullMatrix(Range(0, 3), Range(0, 3))
            if (K0) K0[r * 3 + c] = P[0][r * 4 + c];
            if (K1) K1[r * 3 + c] = P[1][r * 4 + c];
        }
    return YV_OK;
}

int yv_seq_size(const yv_seq* s, int* H, int* W) {
    if (!s || !H || !W) return YV_ERR_INVALID;
    *H = s->H;
    *W = s->W;
    return YV_OK;
}

int yv_seq_read(yv_seq* s, int first, int n, uint8_t* dst, int64_t pitch, int threads) {
    if (!s || !dst || first < 0 || n < 0 || first + n > (int)s->left.size() || pitch < (int64_t)s->H * s->W)
        return YV_ERR_INVALID;
    if (n == 0) return YV_OK;
    return decode_frames(s, first, n, dst, pitch, threads);
}

int yv_seq_upload(yv_seq* s, yv_ctx* ctx, int first, int n, uint8_t* d_dst, int64_t pitch, int threads,
                  void* stream) {
    if (!s || !ctx || !d_dst || first < 0 || n < 0 || first + n > (int)s->left.size() ||
        pitch < (int64_t)s->H * s->W)
        return YV_ERR_INVALID;
    if (n == 0) return YV_OK;
    if (hipSetDevice(yavo::ctx_device(ctx)) != hipSuccess) return YV_ERR_HIP;
    const int k = s->next;
    s->next ^= 1;
    if (s->pending[k] && hipEventSynchronize(s->done[k]) != hipSuccess) return YV_ERR_HIP;
    s->pending[k] = false;
    const size_t bytes = (size_t)pitch * n * (s->stereo ? 2 : 1);
    if (bytes > s->stage_cap[k]) {
        if (s->stage[k]) (void)hipHostFree(s->stage[k]);
        s->stage[k] = nullptr;
        s->stage_cap[k] = 0;
        if (hipHostMalloc(reinterpret_cast<void**>(&s->stage[k]), bytes) != hipSuccess) return YV_ERR_HIP;
        s->stage_cap[k] = bytes;
    }
    if (!s->done[k] && hipEventCreateWithFlags(&s->done[k], hipEventDisableTiming) != hipSuccess) return YV_ERR_HIP;
    const int rc = decode_frames(s, first, n, s->stage[k], pitch, threads);
    if (rc != YV_OK) return rc;
    hipStream_t st = stream ? reinterpret_cast<hipStream_t>(stream) : yavo::ctx_stream(ctx);
    if (hipMemcpyAsync(d_dst, s->stage[k], bytes, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipEventRecord(s->done[k], st) != hipSuccess)
        return YV_ERR_HIP;
    s->pending[k] = true;
    return YV_OK;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// PNG decoding on the GPU: host side (chunk walk, staging, copies, launches)
// ------------------------------------------------------------------------------------------------
struct yv_pngdec {
    yv_ctx* ctx = nullptr;
    int max_images = 0, H = 0, W = 0;
    int64_t raw_pitch = 0;        // inflated image: H rows of 1 + W bytes (+ 64 B of over-read slack), 256-B aligned
    uint8_t* d_raw = nullptr;     // [max_images][raw_pitch]
    int32_t* d_status = nullptr;  // [max_images]
    uint32_t* d_adler = nullptr;  // [max_images] the zlib trailers of the last decode
    uint32_t* d_bad = nullptr;    // images failed since the last yv_pngdec_status
    int check_crc = 1, check_adler = 1;  // yv_pngdec_set_checks
    int n_last = 0;
    hipStream_t last_stream = nullptr;
    // slots of staging: pinned host {streams | offsets | lengths} and the device copy of the streams; four, so that a
    // caller issuing two decodes per step (frames + halo) copies step i + 1's streams while step i's are inflated
    struct Slot {
        uint8_t* h = nullptr;   // pinned: compressed streams (64-B aligned each)
        size_t cap = 0;
        int64_t* h_off = nullptr;
        int32_t* h_len = nullptr;
        uint8_t* d = nullptr;   // device copy of the files
        uint8_t* dg = nullptr;  // their zlib streams, gathered on the device (same offsets)
        size_t dcap = 0;
        yavo::PngPiece* h_pc = nullptr;  // pinned: the IDAT payloads
        yavo::PngPiece* d_pc = nullptr;
        size_t pc_cap = 0;
        hipEvent_t gathered = nullptr;
        int64_t* d_off = nullptr;
        int32_t* d_len = nullptr;
        int32_t* d_crc = nullptr;     // [max_images] a payload CRC failed (gather -> inflate, cleared by the inflate)
        int32_t* h_pre = nullptr;     // pinned [max_images]: kPngErrFile for a file the host could not read / parse
        bool any_pre = false;
        hipEvent_t copied = nullptr;  // the pinned streams are on the device: the host may refill the slot
        hipEvent_t done = nullptr;    // the slot's inflate completed: the device copy may be overwritten
        bool pending = false;
    } slot[4];
    int next = 0;
    hipStream_t copy = nullptr;      // the H2D copies of the streams, beside the kernels
    hipEvent_t last_done = nullptr;  // the last launch's unfilter completed (d_raw / d_status are free)
};

namespace {

// IDAT payloads of one 8-bit grey non-interlaced H x W PNG staged at `base` of the slot: appended to pcs as pieces
// (src = base + payload offset, dst = base + position in the zlib stream); returns the stream's length or -1
int64_t png_idat_pieces(const uint8_t* buf, size_t len, int H, int W, int64_t base, int img,
                        std::vector<yavo::PngPiece>& pcs) {
    PngHeader h;
    if (png_parse(buf, len, h, nullptr, nullptr) != YV_OK) return -1;
    if (h.ctype != 0 || h.depth != 8 || h.interlace != 0 || h.H != H || h.W != W) return -1;
    size_t off = 8;
    int64_t out = 0;
    while (off + 12 <= len) {
        const uint32_t n = be32(buf + off);
        if (n > len - off - 12) return -1;
        const uint8_t* type = buf + off + 4;
        if (!std::memcmp(type, "IDAT", 4)) {
            if (n) pcs.push_back({base + (int64_t)off + 8, base + out, (int32_t)n, (int32_t)img});
            out += n;
        } else if (!std::memcmp(type, "IEND", 4)) {
            break;
        }
        off += 12 + n;
    }
    return out ? out : -1;
}

int slot_reserve(yv_pngdec::Slot& sl, size_t bytes, int n) {
    if (bytes > sl.cap) {
        if (sl.h) (void)hipHostFree(sl.h);
        sl.h = nullptr;
        sl.cap = 0;
        const size_t cap = std::max(bytes + bytes / 4, (size_t)16 << 20);
        if (hipHostMalloc(reinterpret_cast<void**>(&sl.h), cap) != hipSuccess) return YV_ERR_HIP;
        sl.cap = cap;
    }
    if (bytes > sl.dcap) {
        if (sl.pending && hipEventSynchronize(sl.done) != hipSuccess) return YV_ERR_HIP;  // a kernel may still read it
        if (sl.d) (void)hipFree(sl.d);
        if (sl.dg) (void)hipFree(sl.dg);
        sl.d = sl.dg = nullptr;
        sl.dcap = 0;
        const size_t cap = std::max(bytes + bytes / 4, (size_t)16 << 20);
        if (hipMalloc(reinterpret_cast<void**>(&sl.d), cap) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&sl.dg), cap) != hipSuccess)
            return YV_ERR_HIP;
        sl.dcap = cap;
    }
    (void)n;
    return YV_OK;
}

// the slot's piece table holds at least n entries (host: the copies of its last use are done; device: its last
// gather is done)
int slot_reserve_pieces(yv_pngdec::Slot& sl, size_t n) {
    if (n <= sl.pc_cap) return YV_OK;
    if (sl.pending && hipEventSynchronize(sl.done) != hipSuccess) return YV_ERR_HIP;
    if (sl.h_pc) (void)hipHostFree(sl.h_pc);
    if (sl.d_pc) (void)hipFree(sl.d_pc);
    sl.h_pc = nullptr;
    sl.d_pc = nullptr;
    sl.pc_cap = 0;
    const size_t cap = std::max(n + n / 4, (size_t)4096);
    if (hipHostMalloc(reinterpret_cast<void**>(&sl.h_pc), cap * sizeof(yavo::PngPiece)) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&sl.d_pc), cap * sizeof(yavo::PngPiece)) != hipSuccess)
        return YV_ERR_HIP;
    sl.pc_cap = cap;
    return YV_OK;
}

// per-image piece lists -> the slot's pinned table
int slot_set_pieces(yv_pngdec::Slot& sl, const std::vector<std::vector<yavo::PngPiece>>& pcs, int& npc) {
    size_t n = 0;
    for (const auto& v : pcs) n += v.size();
    if (n > (size_t)INT32_MAX) return YV_ERR_INVALID;
    if (slot_reserve_pieces(sl, n) != YV_OK) return YV_ERR_HIP;
    size_t k = 0;
    for (const auto& v : pcs) {
        std::memcpy(sl.h_pc + k, v.data(), v.size() * sizeof(yavo::PngPiece));
        k += v.size();
    }
    npc = (int)n;
    return YV_OK;
}

// the slot's streams are gathered: copy them (and the job table) up, inflate, unfilter
// The copies run on the decoder's copy stream once the slot's last inflate is done with its device buffer; the kernels
// run on st after the copies and after the last launch's kernels (d_raw and d_status are shared).  The host waits only
// for a slot's copies before refilling it (pngdec_next_slot).
int pngdec_launch(yv_pngdec* d, yv_pngdec::Slot& sl, size_t bytes, int n, int npc, uint8_t* d_dst, int64_t pitch,
                  hipStream_t st) {
    hipStream_t cs = d->copy;
    if (sl.pending && hipStreamWaitEvent(cs, sl.done, 0) != hipSuccess) return YV_ERR_HIP;
    if (hipMemcpyAsync(sl.d, sl.h, bytes, hipMemcpyHostToDevice, cs) != hipSuccess ||
        hipMemcpyAsync(sl.d_off, sl.h_off, sizeof(int64_t) * (size_t)n, hipMemcpyHostToDevice, cs) != hipSuccess ||
        hipMemcpyAsync(sl.d_len, sl.h_len, sizeof(int32_t) * (size_t)n, hipMemcpyHostToDevice, cs) != hipSuccess ||
        (npc && hipMemcpyAsync(sl.d_pc, sl.h_pc, sizeof(yavo::PngPiece) * (size_t)npc, hipMemcpyHostToDevice, cs) !=
                    hipSuccess) ||
        (sl.any_pre &&
         hipMemcpyAsync(sl.d_crc, sl.h_pre, sizeof(int32_t) * (size_t)n, hipMemcpyHostToDevice, cs) != hipSuccess) ||
        hipEventRecord(sl.copied, cs) != hipSuccess)
        return YV_ERR_HIP;
    if (npc) yavo::launch_png_gather(sl.d, sl.dg, sl.d_pc, npc, d->check_crc ? sl.d_crc : nullptr, cs);
    if (hipGetLastError() != hipSuccess || hipEventRecord(sl.gathered, cs) != hipSuccess ||
        hipStreamWaitEvent(st, sl.gathered, 0) != hipSuccess ||
        (d->n_last && hipStreamWaitEvent(st, d->last_done, 0) != hipSuccess))
        return YV_ERR_HIP;
    yavo::launch_png_inflate(sl.dg, sl.d_off, sl.d_len, n, d->d_raw, d->raw_pitch, (uint32_t)d->H * (d->W + 1),
                             d->d_status, sl.d_crc, d->check_adler ? d->d_adler : nullptr, st);
    yavo::launch_png_unfilter(d->d_raw, d->raw_pitch, n, d->H, d->W, d_dst, pitch, d->W, d->d_status,
                              d->check_adler ? d->d_adler : nullptr, d->d_bad, st);
    if (hipGetLastError() != hipSuccess || hipEventRecord(sl.done, st) != hipSuccess ||
        hipEventRecord(d->last_done, st) != hipSuccess)
        return YV_ERR_HIP;
    sl.pending = true;
    d->n_last = n;
    d->last_stream = st;
    return YV_OK;
}

yv_pngdec::Slot* pngdec_next_slot(yv_pngdec* d) {
    yv_pngdec::Slot& sl = d->slot[d->next];
    d->next = (d->next + 1) % 4;
    if (sl.pending && hipEventSynchronize(sl.copied) != hipSuccess) return nullptr;
    return &sl;
}

}  // namespace

extern "C" {

int yv_pngdec_create(yv_ctx* ctx, int max_images, int H, int W, yv_pngdec** out) {
    if (!ctx || !out || max_images <= 0 || H < 1 || W < 1 || (int64_t)H * (W + 1) >= (1ll << 31)) return YV_ERR_INVALID;
    *out = nullptr;
    if (hipSetDevice(yavo::ctx_device(ctx)) != hipSuccess) return YV_ERR_HIP;
    yv_pngdec* d = new (std::nothrow) yv_pngdec();
    if (!d) return YV_ERR_INVALID;
    d->ctx = ctx;
    d->max_images = max_images;
    d->H = H;
    d->W = W;
    d->raw_pitch = (((int64_t)H * (W + 1) + 64) + 255) & ~(int64_t)255;
    bool ok = hipMalloc(reinterpret_cast<void**>(&d->d_raw), (size_t)d->raw_pitch * max_images) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&d->d_status), sizeof(int32_t) * (size_t)max_images) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&d->d_adler), sizeof(uint32_t) * (size_t)max_images) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&d->d_bad), sizeof(uint32_t)) == hipSuccess &&
              hipMemset(d->d_bad, 0, sizeof(uint32_t)) == hipSuccess;
    for (auto& sl : d->slot) {
        ok = ok && hipHostMalloc(reinterpret_cast<void**>(&sl.h_off), sizeof(int64_t) * (size_t)max_images) == hipSuccess &&
             hipHostMalloc(reinterpret_cast<void**>(&sl.h_len), sizeof(int32_t) * (size_t)max_images) == hipSuccess &&
             hipHostMalloc(reinterpret_cast<void**>(&sl.h_pre), sizeof(int32_t) * (size_t)max_images) == hipSuccess &&
             hipMalloc(reinterpret_cast<void**>(&sl.d_off), sizeof(int64_t) * (size_t)max_images) == hipSuccess &&
             hipMalloc(reinterpret_cast<void**>(&sl.d_len), sizeof(int32_t) * (size_t)max_images) == hipSuccess &&
             hipMalloc(reinterpret_cast<void**>(&sl.d_crc), sizeof(int32_t) * (size_t)max_images) == hipSuccess &&
             hipMemset(sl.d_crc, 0, sizeof(int32_t) * (size_t)max_images) == hipSuccess &&
             hipEventCreateWithFlags(&sl.copied, hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&sl.gathered, hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&sl.done, hipEventDisableTiming) == hipSuccess;
    }
    ok = ok && hipEventCreateWithFlags(&d->last_done, hipEventDisableTiming) == hipSuccess &&
         hipStreamCreateWithFlags(&d->copy, hipStreamNonBlocking) == hipSuccess;
    if (!ok) {
        yv_pngdec_destroy(d);
        return YV_ERR_HIP;
    }
    *out = d;
    return YV_OK;
}

void yv_pngdec_destroy(yv_pngdec* d) {
    if (!d) return;
    (void)hipSetDevice(yavo::ctx_device(d->ctx));
    if (d->copy) (void)hipStreamSynchronize(d->copy);
    for (auto& sl : d->slot) {
        if (sl.done) {
            (void)hipEventSynchronize(sl.done);
            (void)hipEventDestroy(sl.done);
        }
        if (sl.copied) (void)hipEventDestroy(sl.copied);
        if (sl.gathered) (void)hipEventDestroy(sl.gathered);
        if (sl.h_pc) (void)hipHostFree(sl.h_pc);
        if (sl.d_pc) (void)hipFree(sl.d_pc);
        if (sl.dg) (void)hipFree(sl.dg);
        if (sl.h) (void)hipHostFree(sl.h);
        if (sl.h_off) (void)hipHostFree(sl.h_off);
        if (sl.h_len) (void)hipHostFree(sl.h_len);
        if (sl.h_pre) (void)hipHostFree(sl.h_pre);
        if (sl.d) (void)hipFree(sl.d);
        if (sl.d_off) (void)hipFree(sl.d_off);
        if (sl.d_len) (void)hipFree(sl.d_len);
        if (sl.d_crc) (void)hipFree(sl.d_crc);
    }
    if (d->last_done) (void)hipEventDestroy(d->last_done);
    if (d->copy) (void)hipStreamDestroy(d->copy);
    if (d->d_raw) (void)hipFree(d->d_raw);
    if (d->d_status) (void)hipFree(d->d_status);
    if (d->d_adler) (void)hipFree(d->d_adler);
    if (d->d_bad) (void)hipFree(d->d_bad);
    delete d;
}

int yv_pngdec_decode(yv_pngdec* d, const uint8_t* const* files, const size_t* sizes, int n, uint8_t* d_dst,
                     int64_t pitch, void* stream) {
    if (!d || n < 0 || n > d->max_images || (n > 0 && (!files || !sizes || !d_dst)) || pitch < (int64_t)d->H * d->W)
        return YV_ERR_INVALID;
    if (n == 0) return YV_OK;
    for (int i = 0; i < n; ++i)
        if (!files[i]) return YV_ERR_INVALID;
    if (hipSetDevice(yavo::ctx_device(d->ctx)) != hipSuccess) return YV_ERR_HIP;
    yv_pngdec::Slot* sl = pngdec_next_slot(d);
    if (!sl) return YV_ERR_HIP;
    size_t bytes = 0;
    for (int i = 0; i < n; ++i) bytes += (sizes[i] + 63) & ~(size_t)63;
    if (slot_reserve(*sl, bytes, n) != YV_OK) return YV_ERR_HIP;
    size_t off = 0;
    std::vector<std::vector<yavo::PngPiece>> pcs((size_t)n);
    sl->any_pre = false;
    for (int i = 0; i < n; ++i) {
        std::memcpy(sl->h + off, files[i], sizes[i]);
        int64_t len = png_idat_pieces(sl->h + off, sizes[i], d->H, d->W, (int64_t)off, i, pcs[(size_t)i]);
        sl->h_pre[i] = 0;
        if (len < 0 || len > INT32_MAX) {  // this image fails (kPngErrFile, zero-filled), the others decode
            pcs[(size_t)i].clear();
            len = 0;
            sl->h_pre[i] = yavo::kPngErrFile;
            sl->any_pre = true;
        }
        sl->h_off[i] = (int64_t)off;
        sl->h_len[i] = (int32_t)len;
        off += (sizes[i] + 63) & ~(size_t)63;
    }
    int npc = 0;
    if (slot_set_pieces(*sl, pcs, npc) != YV_OK) return YV_ERR_HIP;
    hipStream_t st = stream ? reinterpret_cast<hipStream_t>(stream) : yavo::ctx_stream(d->ctx);
    return pngdec_launch(d, *sl, off, n, npc, d_dst, pitch, st);
}

int yv_pngdec_set_checks(yv_pngdec* d, int crc, int adler) {
    if (!d) return YV_ERR_INVALID;
    d->check_crc = crc ? 1 : 0;
    d->check_adler = adler ? 1 : 0;
    return YV_OK;
}

int yv_pngdec_status(yv_pngdec* d, int32_t* codes, int* n_bad) {
    if (!d || !n_bad) return YV_ERR_INVALID;
    *n_bad = 0;
    if (d->n_last == 0) return YV_OK;
    if (hipSetDevice(yavo::ctx_device(d->ctx)) != hipSuccess) return YV_ERR_HIP;
    std::vector<int32_t> h((size_t)d->n_last);
    uint32_t bad = 0;
    if (hipStreamSynchronize(d->last_stream) != hipSuccess ||
        hipMemcpy(h.data(), d->d_status, sizeof(int32_t) * h.size(), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&bad, d->d_bad, sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemset(d->d_bad, 0, sizeof(uint32_t)) != hipSuccess)
        return YV_ERR_HIP;
    *n_bad = (int)bad;  // every decode since the last status query, not only the last one
    if (codes) std::memcpy(codes, h.data(), sizeof(int32_t) * h.size());
    return YV_OK;
}

int yv_seq_upload_gpu(yv_seq* s, yv_pngdec* d, int first, int n, uint8_t* d_dst, int64_t pitch, int threads,
                      void* stream) {
    if (!s || first < 0 || n < 0 || first + n > (int)s->left.size()) return YV_ERR_INVALID;
    std::vector<int> frames((size_t)n);
    for (int i = 0; i < n; ++i) frames[(size_t)i] = first + i;
    return yv_seq_upload_gpu_frames(s, d, frames.data(), n, d_dst, pitch, threads, stream);
}

int yv_seq_upload_gpu_frames(yv_seq* s, yv_pngdec* d, const int* frames, int n, uint8_t* d_dst, int64_t pitch,
                             int threads, void* stream) {
    if (!s || !d || !d_dst || n < 0 || (n > 0 && !frames) || s->H != d->H || s->W != d->W) return YV_ERR_INVALID;
    for (int i = 0; i < n; ++i)
        if (frames[i] < 0 || frames[i] >= (int)s->left.size()) return YV_ERR_INVALID;
    const int per = s->stereo ? 2 : 1;
    const int total = n * per;
    if (total > d->max_images || pitch < (int64_t)d->H * d->W) return YV_ERR_INVALID;
    if (n == 0) return YV_OK;
    if (hipSetDevice(yavo::ctx_device(d->ctx)) != hipSuccess) return YV_ERR_HIP;
    yv_pngdec::Slot* sl = pngdec_next_slot(d);
    if (!sl) return YV_ERR_HIP;
    // the threads stat the files, their sizes place them in 64-B aligned regions of the pinned slot, then the threads
    // read each file into its region and gather its IDAT stream to the region's front
    if (threads <= 0) threads = (int)std::min<unsigned>(std::max(1u, std::thread::hardware_concurrency()), 64u);
    threads = std::max(1, std::min(threads, total));
    auto path_of = [&](int k) -> const std::string& {
        return (k % per) ? s->right[frames[k / per]] : s->left[frames[k / per]];
    };
    std::vector<size_t> size((size_t)total), off((size_t)total);
    std::atomic<int> next{0};
    auto run = [&](auto&& job) {
        next = 0;
        auto work = [&]() {
            for (int k; (k = next.fetch_add(1)) < total;) job(k);
        };
        std::vector<std::thread> pool;
        for (int t = 1; t < threads; ++t) pool.emplace_back(work);
        work();
        for (auto& t : pool) t.join();
    };
    // a file that is missing, unreadable, truncated or not an 8-bit grey PNG of the decoder's size fails alone
    // (kPngErrFile, zero-filled, counted by yv_pngdec_status) as cv::imread fails per file; the batch's other images
    // decode
    std::vector<int32_t> pre((size_t)total, 0);
    run([&](int k) {
        struct stat sb;
        if (::stat(path_of(k).c_str(), &sb) != 0 || sb.st_size <= 0) {
            pre[k] = yavo::kPngErrFile;
            size[k] = 0;
            return;
        }
        size[k] = (size_t)sb.st_size;
    });
    size_t bytes = 0;
    for (int k = 0; k < total; ++k) {
        off[k] = bytes;
        bytes += (size[k] + 63) & ~(size_t)63;
    }
    if (slot_reserve(*sl, bytes, total) != YV_OK) return YV_ERR_HIP;
    std::vector<std::vector<yavo::PngPiece>> pcs((size_t)total);
    run([&](int k) {
        sl->h_off[k] = (int64_t)off[k];
        sl->h_len[k] = 0;
        if (pre[k]) return;
        const int fd = ::open(path_of(k).c_str(), O_RDONLY);
        size_t got = 0;
        if (fd >= 0) {
            while (got < size[k]) {
                const ssize_t r = ::read(fd, sl->h + off[k] + got, size[k] - got);
                if (r <= 0) break;
                got += (size_t)r;
            }
            ::close(fd);
        }
        const int64_t len =
            got == size[k] ? png_idat_pieces(sl->h + off[k], size[k], d->H, d->W, (int64_t)off[k], k, pcs[(size_t)k])
                           : -1;
        if (len < 0 || len > INT32_MAX) {
            pcs[(size_t)k].clear();
            pre[k] = yavo::kPngErrFile;
            return;
        }
        sl->h_len[k] = (int32_t)len;
    });
    sl->any_pre = false;
    for (int k = 0; k < total; ++k) {
        sl->h_pre[k] = pre[k];
        sl->any_pre |= pre[k] != 0;
    }
    int npc = 0;
    if (slot_set_pieces(*sl, pcs, npc) != YV_OK) return YV_ERR_HIP;
    hipStream_t st = stream ? reinterpret_cast<hipStream_t>(stream) : yavo::ctx_stream(d->ctx);
    return pngdec_launch(d, *sl, bytes, total, npc, d_dst, pitch, st);
}

int yv_png_write_gray(const char* path, const uint8_t* img, int H, int W, int stride) {
    if (!path || !img || H < 1 || W < 1 || stride < W) return YV_ERR_INVALID;
    // filtered scanlines as cv::imwrite writes them (the reference's tests/epilines.png: every row filter 1 = Sub,
    // zlib header 0x7801): filter byte + W bytes each, then deflate at level 1 with the Z_RLE strategy
    std::vector<uint8_t> raw((size_t)H * (W + 1));
    for (int r = 0; r < H; ++r) {
        const uint8_t* cur = img + (size_t)r * stride;
        uint8_t* o = &raw[(size_t)r * (W + 1)];
        o[0] = 1;
        for (int c = 0; c < W; ++c) o[1 + c] = (uint8_t)(cur[c] - (c ? cur[c - 1] : 0));
    }
    z_stream zs;
    std::memset(&zs, 0, sizeof zs);
    if (deflateInit2(&zs, 1, Z_DEFLATED, 15, 8, Z_RLE) != Z_OK) return YV_ERR_INVALID;
    std::vector<uint8_t> z(deflateBound(&zs, (uLong)raw.size()));
    zs.next_in = raw.data();
    zs.avail_in = (uInt)raw.size();
    zs.next_out = z.data();
    zs.avail_out = (uInt)z.size();
    const int zr = deflate(&zs, Z_FINISH);
    const uLongf zlen = (uLongf)(z.size() - zs.avail_out);
    deflateEnd(&zs);
    if (zr != Z_STREAM_END) return YV_ERR_INVALID;
    FILE* f = std::fopen(path, "wb");
    if (!f) return YV_ERR_INVALID;
    auto be32 = [](uint32_t v, uint8_t* b) {
        b[0] = (uint8_t)(v >> 24); b[1] = (uint8_t)(v >> 16); b[2] = (uint8_t)(v >> 8); b[3] = (uint8_t)v;
    };
    auto chunk = [&](const char* type, const uint8_t* data, uint32_t len) {
        uint8_t hdr[8];
        be32(len, hdr);
        std::memcpy(hdr + 4, type, 4);
        uLong crc = crc32(0L, hdr + 4, 4);
        if (len) crc = crc32(crc, data, len);
        uint8_t tail[4];
        be32((uint32_t)crc, tail);
        std::fwrite(hdr, 1, 8, f);
        if (len) std::fwrite(data, 1, len, f);
        std::fwrite(tail, 1, 4, f);
    };
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    std::fwrite(sig, 1, 8, f);
    uint8_t ihdr[13];
    be32((uint32_t)W, ihdr);
    be32((uint32_t)H, ihdr + 4);
    ihdr[8] = 8;   // bit depth
    ihdr[9] = 0;   // grey
    ihdr[10] = 0;  // deflate
    ihdr[11] = 0;  // adaptive filtering
    ihdr[12] = 0;  // no interlace
    chunk("IHDR", ihdr, 13);
    chunk("IDAT", z.data(), (uint32_t)zlen);
    chunk("IEND", nullptr, 0);
    const bool ok = !std::ferror(f);
    return (std::fclose(f) == 0 && ok) ? YV_OK : YV_ERR_INVALID;
}

int yv_write_kitti_poses(const char* path, const double* poses, int n) {
    if (!path || n < 0 || (n > 0 && !poses)) return YV_ERR_INVALID;
    FILE* f = std::fopen(path, "w");
    if (!f) return YV_ERR_INVALID;
    for (int i = 0; i < n; ++i) {
        const double* p = poses + 7 * (size_t)i;
        double R[9];
        quat_to_R(p, R);
        // T_wc = T_cw^-1: R^T, -R^T t
        double M[12];
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) M[r * 4 + c] = R[c * 3 + r];
            M[r * 4 + 3] = -(R[0 * 3 + r] * p[4] + R[1 * 3 + r] * p[5] + R[2 * 3 + r] * p[6]);
        }
        for (int q = 0; q < 12; ++q) std::fprintf(f, q ? " %.12e" : "%.12e", M[q]);
        std::fputc('\n', f);
    }
    const bool ok = !std::ferror(f);
    return std::fclose(f) == 0 && ok ? YV_OK : YV_ERR_INVALID;
}

int yv_read_kitti_poses(const char* path, double* out, int cap, int* n) {
    if (!path || !n || cap < 0 || (cap > 0 && !out)) return YV_ERR_INVALID;
    FILE* f = std::fopen(path, "r");
    if (!f) return YV_ERR_INVALID;
    int cnt = 0;
    double v[12];
    while (cnt < cap) {
        int got = 0;
        for (; got < 12; ++got)
            if (std::fscanf(f, "%lf", &v[got]) != 1) break;
        if (got == 0) break;
        if (got != 12) {
            std::fclose(f);
            return YV_ERR_INVALID;
        }
        for (int q = 0; q < 12; ++q) out[12 * (size_t)cnt + q] = v[q];
        ++cnt;
    }
    std::fclose(f);
    *n = cnt;
    return YV_OK;
}

}  // extern "C"
