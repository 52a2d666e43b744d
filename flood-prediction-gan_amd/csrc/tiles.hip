// Tile data path: the reference's FloodDataset.__getitem__
// (models/data.py:57-78) -- tifffile.imread of a 9-channel HWC float32 input stack and a 3-channel
// output image, optional np.fliplr -- followed by utils.apply_transformations (models/utils.py:19-67):
// topography channel selection, torchvision Resize(resize, BICUBIC, antialias=True), quadrant crop,
// Normalize(0.5, 0.5).
//
// Host side (C++): a baseline-TIFF reader for the files the reference's pre-processing writes with
// tifffile.imsave(..., planarconfig="contig") (pre_processing/data_pre_processing.py:377-418):
// uncompressed, chunky samples, strips, either byte order, uint8/uint16/float32/float64 samples,
// decoded straight into a caller buffer (a pinned-host staging slot) as float32 HWC.
//
// Device side: the transform of a whole batch of staged raw tiles in two separable passes over only
// the crop window of the resized image -- horizontal (flip, channel selection, column taps) into a
// workspace, then vertical (row taps, normalize) into the output tensor (any strides: the loader
// writes channels-last so the generator's NHWC packer reads it directly).  The antialias bicubic
// taps (the filter torch.nn.functional.interpolate(mode="bicubic", antialias=True) -- what
// torchvision's tensor Resize dispatches to -- uses: Keys a = -0.5, support 2 * in/out when
// downscaling, weights normalized per output index) are computed by the host (floodgan/data.py)
// and passed as tables; width is resampled first, then height, as PyTorch's separable kernel does.
#include <stdio.h>
#include <string.h>

#include <vector>

#include "fg_common.hpp"

namespace {

// ------------------------------------------------------------------------------------------ TIFF

struct Tiff {
    int w = 0, h = 0, spp = 1, bps = 0, fmt = 1, planar = 1, comp = 1, rows_per_strip = 0;
    std::vector<long long> offsets, counts;
};

struct Reader {
    FILE* f = nullptr;
    bool be = false;
    explicit Reader(const char* path) { f = fopen(path, "rb"); }
    ~Reader() {
        if (f) fclose(f);
    }
    bool at(long long off) { return fseeko(f, (off_t)off, SEEK_SET) == 0; }
    bool raw(void* p, size_t n) { return fread(p, 1, n, f) == n; }
    unsigned long long get(int bytes) {
        unsigned char b[8] = {0};
        if (!raw(b, bytes)) return ~0ull;
        unsigned long long v = 0;
        for (int i = 0; i < bytes; ++i) v |= (unsigned long long)b[be ? bytes - 1 - i : i] << (8 * i);
        return v;
    }
};

int type_size(int t) {
    switch (t) {
        case 1: case 2: case 6: case 7: return 1;      // BYTE ASCII SBYTE UNDEFINED
        case 3: case 8: return 2;                        // SHORT SSHORT
        case 4: case 9: case 11: case 13: return 4;      // LONG SLONG FLOAT IFD
        case 5: case 10: case 12: case 16: case 17: case 18: return 8;   // RATIONAL DOUBLE LONG8 ...
        default: return 0;
    }
}

// values of one IFD entry (integer types), reading out-of-line data when it does not fit inline
bool entry_values(Reader& r, int type, unsigned long long count, long long inline_pos, int inline_bytes,
                  std::vector<long long>& out) {
    const int ts = type_size(type);
    if (ts == 0 || count > (1ull << 26)) return false;
    const unsigned long long total = ts * count;
    long long pos = inline_pos;
    if (total > (unsigned long long)inline_bytes) {
        if (!r.at(inline_pos)) return false;
        pos = (long long)r.get(inline_bytes);
    }
    if (!r.at(pos)) return false;
    out.resize(count);
    for (unsigned long long i = 0; i < count; ++i) out[i] = (long long)r.get(ts);
    return true;
}

int parse(Reader& r, Tiff& t) {
    if (!r.f) return fg::fail(FG_ERR_INVALID, "tiff: cannot open file");
    unsigned char hdr[4];
    if (!r.raw(hdr, 4)) return fg::fail(FG_ERR_INVALID, "tiff: short header");
    if (hdr[0] == 'I' && hdr[1] == 'I') r.be = false;
    else if (hdr[0] == 'M' && hdr[1] == 'M') r.be = true;
    else return fg::fail(FG_ERR_INVALID, "tiff: bad byte-order mark");
    const int magic = r.be ? (hdr[2] << 8 | hdr[3]) : (hdr[3] << 8 | hdr[2]);
    const bool big = magic == 43;                         // BigTIFF (tifffile writes it for > 4 GB)
    if (magic != 42 && !big) return fg::fail(FG_ERR_INVALID, "tiff: bad magic %d", magic);
    long long ifd;
    if (big) {
        r.get(2);
        r.get(2);
        ifd = (long long)r.get(8);
    } else {
        ifd = (long long)r.get(4);
    }
    if (!r.at(ifd)) return fg::fail(FG_ERR_INVALID, "tiff: bad IFD offset");
    const unsigned long long n = r.get(big ? 8 : 2);
    if (n == 0 || n > 4096) return fg::fail(FG_ERR_INVALID, "tiff: bad IFD entry count");
    const long long first = ifd + (big ? 8 : 2);
    const int esz = big ? 20 : 12, inl = big ? 8 : 4;
    for (unsigned long long i = 0; i < n; ++i) {
        const long long e = first + (long long)i * esz;
        if (!r.at(e)) return fg::fail(FG_ERR_INVALID, "tiff: truncated IFD");
        const int tag = (int)r.get(2), type = (int)r.get(2);
        const unsigned long long count = r.get(big ? 8 : 4);
        std::vector<long long> v;
        const long long vpos = e + 4 + (big ? 8 : 4);
        switch (tag) {
            case 256: case 257: case 258: case 259: case 262: case 273: case 277: case 278: case 279: case 284:
            case 317: case 322: case 339:
                if (!entry_values(r, type, count, vpos, inl, v) || v.empty())
                    return fg::fail(FG_ERR_INVALID, "tiff: bad value of tag %d", tag);
                break;
            default:
                continue;
        }
        switch (tag) {
            case 256: t.w = (int)v[0]; break;
            case 257: t.h = (int)v[0]; break;
            case 258: t.bps = (int)v[0]; break;
            case 259: t.comp = (int)v[0]; break;
            case 273: t.offsets = v; break;
            case 277: t.spp = (int)v[0]; break;
            case 278: t.rows_per_strip = (int)v[0]; break;
            case 279: t.counts = v; break;
            case 284: t.planar = (int)v[0]; break;
            case 317:
                if (v[0] != 1) return fg::fail(FG_ERR_INVALID, "tiff: predictor %lld not supported", v[0]);
                break;
            case 322: return fg::fail(FG_ERR_INVALID, "tiff: tiled layout not supported (strips only)");
            case 339: t.fmt = (int)v[0]; break;
        }
    }
    if (t.w <= 0 || t.h <= 0 || t.spp <= 0) return fg::fail(FG_ERR_INVALID, "tiff: missing image size");
    if (t.comp != 1) return fg::fail(FG_ERR_INVALID, "tiff: compression %d not supported (uncompressed only)", t.comp);
    if (t.spp > 1 && t.planar != 1) return fg::fail(FG_ERR_INVALID, "tiff: planar (separate) layout not supported");
    const bool ok = (t.fmt == 1 && (t.bps == 8 || t.bps == 16)) || (t.fmt == 3 && (t.bps == 32 || t.bps == 64));
    if (!ok) return fg::fail(FG_ERR_INVALID, "tiff: sample format %d / %d bits not supported", t.fmt, t.bps);
    if (t.offsets.empty() || t.offsets.size() != t.counts.size())
        return fg::fail(FG_ERR_INVALID, "tiff: missing strip offsets / byte counts");
    if (t.rows_per_strip <= 0 || t.rows_per_strip > t.h) t.rows_per_strip = t.h;
    return 0;
}

// sample -> float, host byte order fix-up
template <typename T>
inline T swap_bytes(T v) {
    unsigned char* b = reinterpret_cast<unsigned char*>(&v);
    for (size_t i = 0; i < sizeof(T) / 2; ++i) {
        const unsigned char c = b[i];
        b[i] = b[sizeof(T) - 1 - i];
        b[sizeof(T) - 1 - i] = c;
    }
    return v;
}

template <typename T>
void convert(const unsigned char* src, size_t n, bool swap, float* dst) {
    for (size_t i = 0; i < n; ++i) {
        T v;
        memcpy(&v, src + i * sizeof(T), sizeof(T));
        if (swap) v = swap_bytes(v);
        dst[i] = (float)v;
    }
}

// ------------------------------------------------------------------------------------------ kernels

// horizontal pass: tmp[n][y][j][o] = sum_k wx[c0 + j][k] * src[n][y][flip(x0(c0 + j) + k)][chan[o]]
__global__ void tile_hpass_kernel(const fg_tile_batch B, int rows) {
    const long long total = (long long)B.n * rows * B.out_w;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int j = (int)(idx % B.out_w);
        const long long t = idx / B.out_w;
        const int y = (int)(t % rows);
        const int n = (int)(t / rows);
        const int c0 = B.crop ? B.crop[2 * n + 1] : 0;
        const int yy = y + (B.crop ? B.row_lo[n] : 0);
        const int xo = c0 + j;
        const int x0 = B.x_idx0[xo];
        const float* wt = B.x_w + (size_t)xo * B.x_taps;
        const float* row = B.src + (size_t)n * B.tile_stride + (size_t)yy * B.w_in * B.c_src;
        const bool flip = B.flip && B.flip[n];
        float acc[FG_TILE_MAX_CH];
#pragma unroll
        for (int o = 0; o < FG_TILE_MAX_CH; ++o) acc[o] = 0.f;
        for (int k = 0; k < B.x_taps; ++k) {
            const float w = wt[k];
            if (w == 0.f) continue;
            int x = x0 + k;
            if (flip) x = B.w_in - 1 - x;
            const float* px = row + (size_t)x * B.c_src;
#pragma unroll
            for (int o = 0; o < FG_TILE_MAX_CH; ++o)
                if (o < B.c_out) acc[o] += w * px[B.chan[o]];
        }
        float* dst = B.tmp + ((size_t)(n * rows + y) * B.out_w + j) * B.c_out;
#pragma unroll
        for (int o = 0; o < FG_TILE_MAX_CH; ++o)
            if (o < B.c_out) dst[o] = acc[o];
    }
}

// vertical pass + Normalize(0.5, 0.5): dst[n][o][i][j] = (sum_k wy[r0 + i][k] * tmp[n][y0 - lo + k][j][o] - 0.5) / 0.5
__global__ void tile_vpass_kernel(const fg_tile_batch B, int rows) {
    const long long total = (long long)B.n * B.out_h * B.out_w;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * blockDim.x) {
        const int j = (int)(idx % B.out_w);
        const long long t = idx / B.out_w;
        const int i = (int)(t % B.out_h);
        const int n = (int)(t / B.out_h);
        const int r0 = B.crop ? B.crop[2 * n] : 0;
        const int lo = B.crop ? B.row_lo[n] : 0;
        const int yo = r0 + i;
        const int y0 = B.y_idx0[yo] - lo;
        const float* wt = B.y_w + (size_t)yo * B.y_taps;
        float acc[FG_TILE_MAX_CH];
#pragma unroll
        for (int o = 0; o < FG_TILE_MAX_CH; ++o) acc[o] = 0.f;
        for (int k = 0; k < B.y_taps; ++k) {
            const float w = wt[k];
            if (w == 0.f) continue;
            const float* px = B.tmp + ((size_t)(n * rows + y0 + k) * B.out_w + j) * B.c_out;
#pragma unroll
            for (int o = 0; o < FG_TILE_MAX_CH; ++o)
                if (o < B.c_out) acc[o] += w * px[o];
        }
        float* d = B.dst.ptr + n * B.dst.sn + i * B.dst.sy + j * B.dst.sx;
#pragma unroll
        for (int o = 0; o < FG_TILE_MAX_CH; ++o)
            if (o < B.c_out) d[o * B.dst.sc] = (acc[o] - 0.5f) / 0.5f;
    }
}

}  // namespace

FG_API int fg_tiff_probe(const char* path, int* height, int* width, int* channels, int* sample_code) {
    if (!path) return fg::fail(FG_ERR_INVALID, "fg_tiff_probe: null path");
    Reader r(path);
    Tiff t;
    const int e = parse(r, t);
    if (e) return e;
    if (height) *height = t.h;
    if (width) *width = t.w;
    if (channels) *channels = t.spp;
    if (sample_code) *sample_code = t.fmt * 100 + t.bps;
    return 0;
}

FG_API int fg_tiff_read(const char* path, float* dst, long long capacity) {
    if (!path || !dst) return fg::fail(FG_ERR_INVALID, "fg_tiff_read: null argument");
    Reader r(path);
    Tiff t;
    const int e = parse(r, t);
    if (e) return e;
    const long long n = (long long)t.h * t.w * t.spp;
    if (capacity < n) return fg::fail(FG_ERR_INVALID, "fg_tiff_read: capacity %lld < %lld samples", capacity, n);
    const int bytes = t.bps / 8;
    const long long row_bytes = (long long)t.w * t.spp * bytes;
    const int nstrips = (t.h + t.rows_per_strip - 1) / t.rows_per_strip;
    if ((int)t.offsets.size() < nstrips) return fg::fail(FG_ERR_INVALID, "fg_tiff_read: %d strips listed, %d needed",
                                                         (int)t.offsets.size(), nstrips);
    const bool swap = r.be;      // hosts are little endian (x86-64)
    std::vector<unsigned char> buf;
    for (int s = 0; s < nstrips; ++s) {
        const int rows = std::min(t.rows_per_strip, t.h - s * t.rows_per_strip);
        const long long need = rows * row_bytes;
        if (t.counts[s] < need) return fg::fail(FG_ERR_INVALID, "fg_tiff_read: strip %d short", s);
        float* out = dst + (long long)s * t.rows_per_strip * t.w * t.spp;
        if (t.fmt == 3 && t.bps == 32 && !swap) {        // the dataset's own format: straight into dst
            if (!r.at(t.offsets[s]) || !r.raw(out, (size_t)need))
                return fg::fail(FG_ERR_INVALID, "fg_tiff_read: read error in strip %d", s);
            continue;
        }
        buf.resize((size_t)need);
        if (!r.at(t.offsets[s]) || !r.raw(buf.data(), (size_t)need))
            return fg::fail(FG_ERR_INVALID, "fg_tiff_read: read error in strip %d", s);
        const size_t cnt = (size_t)(need / bytes);
        if (t.fmt == 3 && t.bps == 32) convert<float>(buf.data(), cnt, swap, out);
        else if (t.fmt == 3) convert<double>(buf.data(), cnt, swap, out);
        else if (t.bps == 8) convert<unsigned char>(buf.data(), cnt, false, out);
        else convert<unsigned short>(buf.data(), cnt, swap, out);
    }
    return 0;
}

FG_API int fg_tile_transform(const fg_tile_batch* b, hipStream_t stream) {
    if (!b || !b->src || !b->tmp || !b->dst.ptr || !b->x_idx0 || !b->x_w || !b->y_idx0 || !b->y_w)
        return fg::fail(FG_ERR_INVALID, "fg_tile_transform: null argument");
    const fg_tile_batch& B = *b;
    if (B.n <= 0 || B.h_in <= 0 || B.w_in <= 0 || B.c_src <= 0 || B.c_out <= 0 || B.c_out > FG_TILE_MAX_CH ||
        B.out_h <= 0 || B.out_w <= 0 || B.x_taps <= 0 || B.y_taps <= 0 || B.rows <= 0 || B.rows > B.h_in ||
        B.tile_stride < (long long)B.h_in * B.w_in * B.c_src)
        return fg::fail(FG_ERR_INVALID, "fg_tile_transform: bad sizes");
    for (int o = 0; o < B.c_out; ++o)
        if (B.chan[o] < 0 || B.chan[o] >= B.c_src) return fg::fail(FG_ERR_INVALID, "fg_tile_transform: channel map");
    if (B.crop && !B.row_lo) return fg::fail(FG_ERR_INVALID, "fg_tile_transform: crop needs row_lo");
    const long long h_work = (long long)B.n * B.rows * B.out_w;
    hipLaunchKernelGGL(tile_hpass_kernel, dim3(fg::blocks_for(h_work, 256, 16384)), dim3(256), 0, stream, B, B.rows);
    int e = fg::launched("tile_hpass");
    if (e) return e;
    const long long v_work = (long long)B.n * B.out_h * B.out_w;
    hipLaunchKernelGGL(tile_vpass_kernel, dim3(fg::blocks_for(v_work, 256, 16384)), dim3(256), 0, stream, B, B.rows);
    return fg::launched("tile_vpass");
}
