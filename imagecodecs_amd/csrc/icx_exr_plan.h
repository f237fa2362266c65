// icx_exr_plan.h -- the host side of the OpenEXR read (icx_exr.hip) and the per-pixel gather the
// convert kernel runs, shared with the CPU emulator (tests/emu/exr_emu.cpp). See icx_exr.hip.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "icx_exr_core.h"

namespace icx {

namespace {

enum : int {
    kExrOk = 0, kExrInvalidMagic = -1, kExrInvalidVersion = -2, kExrInvalidArgument = -3, kExrInvalidData = -4,
    kExrUnsupportedFormat = -8, kExrInvalidHeader = -9, kExrUnsupportedFeature = -10
};
constexpr int64_t kThresh = 1024 * 8192;  // TINYEXR_DIMENSION_THRESHOLD (:3628)
constexpr int kIntMax = 0x7fffffff;

int32_t rd32(const uint8_t* p) { int32_t v; std::memcpy(&v, p, 4); return v; }
uint32_t rdu32(const uint8_t* p) { uint32_t v; std::memcpy(&v, p, 4); return v; }
uint64_t rd64(const uint8_t* p) { uint64_t v; std::memcpy(&v, p, 8); return v; }

}  // namespace

// Per chunk: where its pixel bytes are and how they are laid out (DecodePixelData's arguments).
struct ExrChunk {
    int64_t src;        // file offset of the chunk's pixel data
    int64_t len;        // its size (data_len)
    int64_t scratch;    // byte offset of the decompressed bytes in the scratch (modes 1-3)
    int64_t out_len;    // width * lines * pixel_data_size
    int64_t produced;   // bytes the decompressor produced (device)
    int32_t mode;       // 0 pixel bytes are the file's (NONE, or stored raw), 1 ZIP, 2 RLE, 3 PIZ
    int32_t width;      // samples per line of this chunk
    int32_t lines;      // lines it holds
    int32_t piz_len;    // PIZ: the Huffman data's length field
    int64_t piz_bitmap; // PIZ: file offset of the range bitmap's first byte (byte minNonZero)
    int64_t piz_huf;    // PIZ: file offset of the Huffman data
    int64_t piz_work;   // PIZ: scratch offset of the channel planes (out_len); the long-code lists
                        // (PizWork) come from a fixed pool, one per resident k_exr_piz workgroup
    int32_t piz_mnmx;   // PIZ: minNonZero | maxNonZero << 16
    int32_t img;        // batch reads: the chunk's image (its failure flag)
    int64_t base;       // batch reads: its file's device address minus the first file's (k_exr_unpack)
};

struct ExrPlan {
    int w = 0, h = 0, nch = 0, pds = 0, comp = 0, tiled = 0, tx = 0, ty = 0, ntx = 0, line_order = 0;
    int levels = 1;  // tiled: levels decoded (mip- / rip-mapped files: all of them; level 0 is output)
    int src[4] = {-1, -1, -1, -1};  // channel of R, G, B, A (-1: A = 1.0)
    std::vector<int32_t> type, offs;
    std::vector<ExrChunk> chunks;
    std::vector<int2> map;  // scanline: per row {chunk, line}; tiled: per tile position {chunk, 0}; -1: none
    std::vector<int32_t> tile_h;  // tiled: the lines each chunk decoded (DecodeTiledPixelData's height)
    int64_t scratch = 0;
};

// Tiled levels (PrecalculateTileInfo / InitTileOffsets / LevelSize, tinyexr.h:4950-4979,
// :5582-5802): per level in offset-table order its (lx, ly) and tiles across / down.
struct ExrLevel {
    int lx, ly;
    int64_t nx, ny;
};
inline int exr_level_size(int64_t top, int level, int rounding) {  // LevelSize (:4967-4979)
    const int64_t b = (int64_t)1 << level;
    int64_t ls = top / b;
    if (rounding == 1 && ls * b < top) ls += 1;
    return (int)std::max<int64_t>(ls, 1);
}
inline int exr_log2(int64_t x, int rounding) {  // FloorLog2 / CeilLog2 (:5582-5614)
    int y = 0, r = 0;
    while (x > 1) {
        if (x & 1) r = 1;
        ++y;
        x >>= 1;
    }
    return y + (rounding == 1 ? r : 0);
}
inline bool exr_levels(int64_t W, int64_t H, int mode, int rounding, int64_t tx, int64_t ty, std::vector<ExrLevel>& L) {
    int nxl, nyl;
    if (mode == 0) nxl = nyl = 1;
    else if (mode == 1) nxl = nyl = exr_log2(std::max(W, H), rounding) + 1;
    else if (mode == 2) { nxl = exr_log2(W, rounding) + 1; nyl = exr_log2(H, rounding) + 1; }
    else return false;  // CalculateNumXLevels: -1
    std::vector<int64_t> ntx(nxl), nty(nyl);
    for (int i = 0; i < nxl; ++i) {  // CalculateNumTiles (:5692-5706)
        const int64_t l = exr_level_size(W, i, rounding);
        if (l > (int64_t)kIntMax - tx + 1) return false;
        ntx[i] = (l + tx - 1) / tx;
    }
    for (int i = 0; i < nyl; ++i) {
        const int64_t l = exr_level_size(H, i, rounding);
        if (l > (int64_t)kIntMax - ty + 1) return false;
        nty[i] = (l + ty - 1) / ty;
    }
    L.clear();
    if (mode != 2) {
        for (int l = 0; l < nxl; ++l) L.push_back({l, l, ntx[l], nty[l]});
    } else {
        for (int ly = 0; ly < nyl; ++ly)
            for (int lx = 0; lx < nxl; ++lx) L.push_back({lx, ly, ntx[lx], nty[ly]});
    }
    return true;
}

// DecompressPiz's range header (:3232-3314): where it returns false the chunk fails (-1);
// otherwise its fields go to the chunk. inLen == tmpBufSize (stored raw) is mode 0 before this.
inline bool exr_piz_head(const uint8_t* buf, int64_t size, ExrChunk& c) {
    const int64_t in_len = c.len, src = c.src;
    if (in_len < 4) return false;
    const uint32_t mn = buf[src] | buf[src + 1] << 8, mx = buf[src + 2] | buf[src + 3] << 8;
    if (mx >= 8192) return false;  // BITMAP_SIZE
    int64_t rd = 4;
    if (mn <= mx) {
        if ((int64_t)(mx - mn + 1) + rd > in_len) return false;
        rd += mx - mn + 1;
    } else if (!(mn == 8191 && mx == 0)) {
        return false;
    }
    if (rd + 4 > in_len) return false;
    const int32_t length = rd32(buf + src + rd);
    rd += 4;
    if ((uint64_t)(rd + (int64_t)length) > (uint64_t)in_len) return false;  // size_t((ptr - inPtr) + length)
    c.piz_mnmx = (int32_t)(mn | mx << 16);
    c.piz_bitmap = src + 4;
    c.piz_huf = src + rd;
    c.piz_len = length;
    (void)size;
    return true;
}

// ParseEXRVersionFromMemory + ParseEXRHeader + ConvertHeader + DecodeEXRImage's table reading +
// DecodeChunk's per-chunk checks (tinyexr.h:8927-8982, :4441-4940, :6005-6199, :5163-5542).
inline int exr_plan(const uint8_t* buf, int64_t size, ExrPlan& P) {
    if (size < 8) return kExrInvalidData;
    static const uint8_t kMagic[4] = {0x76, 0x2F, 0x31, 0x01};
    if (std::memcmp(buf, kMagic, 4) != 0) return kExrInvalidMagic;
    if (buf[4] != 2) return kExrInvalidVersion;
    const bool tiled_v = buf[5] & 2, multipart = buf[5] & 0x10, non_image = buf[5] & 0x8;
    struct Ch { std::string name; int32_t type; };
    std::vector<Ch> chans;
    int32_t dw[4] = {0, 0, 0, 0}, chunk_count = 0, comp = -1, line_order = 0;
    int64_t tile_x = -1, tile_y = -1;
    int tile_mode = -1, tile_round = -1, tiled = 0;
    std::string type_attr;
    unsigned have = 0;  // required attributes seen
    enum { kComp = 1, kChans = 2, kDW = 4, kDisp = 8, kLO = 16, kPAR = 32, kSWC = 64, kSWW = 128, kName = 256, kType = 512 };
    int ret = kExrOk;
    int64_t p = 8, rem = size - 8;
    for (int nattr = 0; nattr < 1024; ++nattr) {  // TINYEXR_MAX_HEADER_ATTRIBUTES
        if (rem == 0) { ret = kExrInvalidData; break; }
        if (buf[p] == 0) { --rem; break; }
        // ReadAttribute (:1069-1135)
        const char* m = (const char*)buf + p;
        const int64_t nlen = (int64_t)strnlen(m, (size_t)rem);
        if (nlen == rem) { ret = kExrInvalidData; break; }
        const std::string name(m, (size_t)nlen);
        const int64_t r2 = rem - nlen - 1;
        const int64_t tlen = (int64_t)strnlen(m + nlen + 1, (size_t)r2);
        if (tlen == r2) { ret = kExrInvalidData; break; }
        const std::string typ(m + nlen + 1, (size_t)tlen);
        const int64_t r3 = r2 - tlen - 1;
        if (r3 < 4) { ret = kExrInvalidData; break; }
        const uint32_t dlen = rdu32(buf + p + nlen + 1 + tlen + 1);
        std::vector<uint8_t> data;
        int64_t msize;
        if (dlen == 0) {
            if (typ != "string") { ret = kExrInvalidData; break; }
            data.assign(1, 0);
            msize = nlen + 1 + tlen + 1 + 4;
        } else {
            if ((uint64_t)(r3 - 4) < dlen) { ret = kExrInvalidData; break; }
            const uint8_t* d = buf + p + nlen + 1 + tlen + 1 + 4;
            data.assign(d, d + dlen);
            msize = nlen + 1 + tlen + 1 + 4 + dlen;
        }
        p += msize;
        rem -= msize;
        if ((tiled_v || multipart || non_image) && name == "tiles") {
            if (data.size() != 9) { ret = kExrInvalidData; break; }
            const uint32_t xs = rdu32(data.data()), ys = rdu32(data.data() + 4);
            if (xs > (uint32_t)kIntMax || ys > (uint32_t)kIntMax) { ret = kExrUnsupportedFormat; break; }
            tile_x = xs;
            tile_y = ys;
            tile_mode = data[8] & 3;
            tile_round = (data[8] >> 4) & 1;
            tiled = 1;
        } else if (name == "compression") {
            if (data[0] > 4) { ret = kExrUnsupportedFormat; break; }  // unknown / ZFP not built (:4568-4601)
            comp = data[0];
            have |= kComp;
        } else if (name == "channels") {  // ReadChannelInfo (:1226-1272)
            size_t q = 0;
            bool ok = true;  // (a second "channels" attribute appends, as tinyexr's push_back does)
            for (;;) {
                if (q >= data.size()) { ok = false; break; }
                if (data[q] == 0) break;
                size_t z = q;
                while (z < data.size() && data[z]) ++z;
                if (z >= data.size()) { ok = false; break; }
                Ch c;
                c.name.assign((const char*)data.data() + q, z - q);
                q = z + 1;
                if (q + 16 >= data.size()) { ok = false; break; }
                c.type = rd32(data.data() + q);
                chans.push_back(c);
                q += 16;
            }
            if (!ok || chans.empty()) { ret = kExrInvalidData; break; }
            have |= kChans;
        } else if (name == "dataWindow") {
            if (data.size() >= 16) {
                for (int k = 0; k < 4; ++k) dw[k] = rd32(data.data() + 4 * k);
                have |= kDW;
            }
        } else if (name == "displayWindow") {
            if (data.size() >= 16) have |= kDisp;
        } else if (name == "lineOrder") {
            if (!data.empty()) { line_order = data[0]; have |= kLO; }
        } else if (name == "pixelAspectRatio") {
            if (data.size() >= 4) have |= kPAR;
        } else if (name == "screenWindowCenter") {
            if (data.size() >= 8) have |= kSWC;
        } else if (name == "screenWindowWidth") {
            if (data.size() >= 4) have |= kSWW;
        } else if (name == "chunkCount") {
            if (data.size() >= 4) chunk_count = rd32(data.data());
        } else if (name == "name") {
            if (!data.empty() && data[0]) have |= kName;
        } else if (name == "type") {
            if (!data.empty() && data[0]) {
                type_attr.assign((const char*)data.data(), strnlen((const char*)data.data(), data.size()));
                have |= kType;
            }
        }
    }
    if (ret == kExrOk) {
        unsigned need = kComp | kChans | kDW | kDisp | kLO | kPAR | kSWC | kSWW;
        if (multipart || non_image) need |= kName | kType;
        if ((have & need) != need) ret = kExrInvalidHeader;
    }
    if ((type_attr == "scanlineimage" && tiled) || ((type_attr == "tiledimage" || type_attr == "deeptile") && !tiled))
        ret = kExrInvalidHeader;  // ConvertHeader (:4829-4876), whatever ParseEXRHeader returned
    if (ret != kExrOk) return ret;
    const int64_t header_len = (size - 8) - rem;
    // LoadEXRFromMemory / DecodeEXRImage (no multi-part / deep rejection here: only LoadEXR has
    // one, :6268-6270; the flags reach only ReconstructTileOffsets below)
    if (size <= 8) return kExrInvalidArgument;
    int64_t marker = header_len + 8;
    const int nsb = comp == 3 ? 16 : comp == 4 ? 32 : 1;
    if (dw[2] < dw[0] || (int64_t)dw[2] - dw[0] == kIntMax) return kExrInvalidData;
    const int64_t W = (int64_t)dw[2] - dw[0] + 1;
    if (dw[3] < dw[1] || (int64_t)dw[3] - dw[1] == kIntMax) return kExrInvalidData;
    const int64_t H = (int64_t)dw[3] - dw[1] + 1;
    if (W > kThresh || H > kThresh) return kExrInvalidData;
    std::vector<uint64_t> offsets;
    std::vector<ExrLevel> levels;
    auto read_offsets = [&](int64_t n) -> bool {
        // (a count the file cannot hold fails before any allocation: tinyexr's loop runs off the
        // buffer with the same kExrInvalidData; a bad_alloc here would cross the C ABI)
        if (n < 0 || n > (size - marker) / 8) return false;
        offsets.resize((size_t)n);
        for (int64_t k = 0; k < n; ++k) {
            if (marker + 8 >= size) return false;
            const uint64_t o = rd64(buf + marker);
            if (o >= (uint64_t)size) return false;
            marker += 8;
            offsets[(size_t)k] = o;
        }
        return true;
    };
    if (tiled) {
        if (tile_x > kThresh || tile_y > kThresh) return kExrInvalidData;
        if (tile_x == 0 || tile_y == 0) return kExrInvalidData;  // (tinyexr divides by it)
        if (!exr_levels(W, H, tile_mode, tile_round, tile_x, tile_y, levels)) return kExrInvalidData;
        int64_t nblocks = 0;
        for (const ExrLevel& l : levels) nblocks += l.nx * l.ny;
        if (chunk_count > 0 && chunk_count != nblocks) return kExrInvalidData;
        if (!read_offsets(nblocks)) return kExrInvalidData;
        if (std::find(offsets.begin(), offsets.end(), 0ull) != offsets.end()) {
            // ReconstructTileOffsets (:5867-5974): each chunk after the table goes to the place its
            // own header names (places none names keep the table's). The version flags reach it
            // (:6101-6103): a multi-part chunk's 4-byte part number is skipped (the offset kept is
            // the one before it), a deep chunk's two int64 sizes and payloads are skipped.
            const int nxl = tile_mode == 2 ? levels.back().lx + 1 : (int)levels.size();
            const int nyl = tile_mode == 2 ? levels.back().ly + 1 : (int)levels.size();
            std::vector<int64_t> lbase(levels.size() + 1, 0);
            for (size_t l = 0; l < levels.size(); ++l) lbase[l + 1] = lbase[l] + levels[l].nx * levels[l].ny;
            int64_t mk = marker;
            for (int64_t k = 0; k < nblocks; ++k) {
                const int64_t here = mk;
                if (multipart) {
                    if (mk < 0 || mk + 4 >= size) return kExrInvalidData;
                    mk += 4;
                }
                if (mk < 0 || mk + 16 >= size) return kExrInvalidData;
                const int32_t tx_ = rd32(buf + mk), ty_ = rd32(buf + mk + 4), lx = rd32(buf + mk + 8), ly = rd32(buf + mk + 12);
                mk += 16;
                if (non_image) {
                    if (mk + 16 >= size) return kExrInvalidData;
                    uint64_t pot, ps;
                    std::memcpy(&pot, buf + mk, 8);
                    std::memcpy(&ps, buf + mk + 8, 8);
                    mk = (int64_t)((uint64_t)mk + 16u + pot + ps + 8u);
                    if (mk >= size || mk < 0) return kExrInvalidData;
                } else {
                    if (mk + 4 >= size) return kExrInvalidData;
                    mk += 4 + (int64_t)rd32(buf + mk);
                }
                if (lx < 0 || ly < 0 || tx_ < 0 || ty_ < 0) return kExrInvalidData;  // isValidTile (:5814-5865)
                if (tile_mode == 0 && (lx != 0 || ly != 0)) return kExrInvalidData;
                if (tile_mode != 0 && (lx >= nxl || ly >= nyl)) return kExrInvalidData;
                const int64_t li = tile_mode == 0 ? 0 : tile_mode == 1 ? lx : (int64_t)lx + (int64_t)ly * nxl;  // LevelIndex
                if (li >= (int64_t)levels.size()) return kExrInvalidData;
                if (ty_ >= levels[li].ny || tx_ >= levels[li].nx) return kExrInvalidData;
                offsets[(size_t)(lbase[li] + ty_ * levels[li].nx + tx_)] = (uint64_t)here;
            }
        }
    } else {
        const int64_t nb = chunk_count > 0 ? chunk_count : (H + nsb - 1) / nsb;
        if (!read_offsets(nb)) return kExrInvalidData;
        if (std::find(offsets.begin(), offsets.end(), 0ull) != offsets.end()) {  // ReconstructLineOffsets (:5544-5580)
            int64_t mk = marker;
            for (int64_t k = 0; k < nb; ++k) {
                if (mk + 8 >= size) return kExrInvalidData;
                const uint32_t dl = rdu32(buf + mk + 4);
                if (dl >= (uint64_t)size) return kExrInvalidData;
                offsets[(size_t)k] = (uint64_t)mk;
                mk += (int64_t)dl + 8;
            }
        }
    }
    // ComputeChannelLayout (:4321-4350)
    P.type.clear();
    P.offs.clear();
    int pds = 0;
    for (const Ch& c : chans) {
        if (c.type < 0 || c.type > 2) return kExrInvalidData;
        P.type.push_back(c.type);
        P.offs.push_back(pds);
        pds += c.type == 1 ? 2 : 4;
    }
    P.w = (int)W;
    P.h = (int)H;
    P.nch = (int)chans.size();
    P.pds = pds;
    P.comp = comp;
    P.tiled = tiled;
    P.line_order = line_order;
    P.chunks.clear();
    P.scratch = 0;
    auto add_chunk = [&](int64_t src, int64_t len, int width, int lines) -> int {
        ExrChunk c{};
        c.src = src;
        c.len = len;
        c.width = width;
        c.lines = lines;
        c.out_len = (int64_t)width * lines * pds;
        c.mode = comp == 0 ? 0 : (len == c.out_len ? 0 : (comp == 1 ? 2 : comp == 4 ? 3 : 1));
        if (comp == 0 && len < c.out_len) return -1;  // "Insufficient data size" (:4192-4196)
        if (comp != 0 && c.out_len == 0) return -1;   // dstLen == 0 (:3801, :3943); PIZ: #90 (:3643)
        if (c.mode == 3 && !exr_piz_head(buf, size, c)) return -1;
        if (c.mode != 0) {
            c.scratch = P.scratch;
            P.scratch += (c.out_len + 15) / 16 * 16;
        }
        if (c.mode == 3) {  // the channel planes, then the long-code lists
            c.piz_work = P.scratch;
            P.scratch += (c.out_len + 15) / 16 * 16;
        }
        P.chunks.push_back(c);
        return (int)P.chunks.size() - 1;
    };
    if (tiled) {
        const int64_t ntx = levels[0].nx, nty = levels[0].ny;
        P.tx = (int)tile_x;
        P.ty = (int)tile_y;
        P.ntx = (int)ntx;
        P.levels = (int)levels.size();
        P.map.assign((size_t)(ntx * nty), make_int2(-1, 0));
        P.tile_h.clear();
        std::vector<int2> coords;
        // DecodeChunk's level loops (:5282-5354): every level's tiles are decoded and checked
        // (DecodeTiledLevel :4981-5161); the RGBA output takes level 0, the first ntx * nty
        // chunks (:6789-6828)
        size_t k = 0;
        for (const ExrLevel& L : levels) {
            const int64_t lw = exr_level_size(W, L.lx, tile_round), lh = exr_level_size(H, L.ly, tile_round);
            for (int64_t t = 0; t < L.nx * L.ny; ++t, ++k) {
                const int64_t o = (int64_t)offsets[k];
                if (o + 20 > size) return kExrInvalidData;
                const int64_t dsz = size - (o + 20);
                const int32_t cx = rd32(buf + o), cy = rd32(buf + o + 4), lx = rd32(buf + o + 8), ly = rd32(buf + o + 12);
                if (lx != L.lx || ly != L.ly) return kExrInvalidData;
                const int32_t dlen = rd32(buf + o + 16);
                if (dlen < 2 || (int64_t)dlen > dsz) return kExrInvalidData;
                // DecodeTiledPixelData (:4283-4319), in the level's size, tinyexr's int arithmetic
                // (32-bit products: a damaged coordinate wraps as in the reference build)
                auto m32 = [](int64_t a, int64_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); };
                if (m32(tile_x, cx) > lw || m32(tile_y, cy) > lh) return kExrInvalidData;
                const int tw = (m32((uint32_t)cx + 1u, tile_x) >= lw) ? (int32_t)((uint32_t)lw - (uint32_t)m32(cx, tile_x)) : (int)tile_x;
                const int th = (m32((uint32_t)cy + 1u, tile_y) >= lh) ? (int32_t)((uint32_t)lh - (uint32_t)m32(cy, tile_y)) : (int)tile_y;
                const int ci = add_chunk(o + 20, dlen, tw, th);
                if (ci < 0) return kExrInvalidData;
                P.tile_h.push_back(th);
                if (k < (size_t)(ntx * nty)) coords.push_back(make_int2(cx, cy));
            }
        }
        // the RGBA loop (:6789-6828) visits level 0's tiles in order: the last tile at a position
        // wins; negative origins are past the image as size_t
        for (size_t k = 0; k < coords.size(); ++k) {
            const int64_t cx = coords[k].x, cy = coords[k].y;
            if (cx < 0 || cy < 0 || cx >= ntx || cy >= nty) continue;
            P.map[(size_t)(cy * ntx + cx)] = make_int2((int)k, 0);
        }
    } else {
        P.map.assign((size_t)H, make_int2(-1, 0));
        for (size_t y = 0; y < offsets.size(); ++y) {  // DecodeChunk's scanline loop (:5409-5496)
            const int64_t o = (int64_t)offsets[y];
            if (o + 8 > size) return kExrInvalidData;
            const int64_t dsz = size - (o + 8);
            const int32_t line_no = rd32(buf + o), dlen = rd32(buf + o + 4);
            if (dlen < 0 || (int64_t)dlen > dsz) return kExrInvalidData;
            if (line_no > (2 << 20) || line_no < -(2 << 20) || dlen == 0) return kExrInvalidData;
            const int64_t end = std::min<int64_t>((int64_t)line_no + nsb, (int64_t)dw[3] + 1);
            const int64_t nl = end - line_no;
            if (nl <= 0) return kExrInvalidData;
            const int64_t lno = (int64_t)line_no - dw[1];
            if (lno < 0 || lno > kIntMax) return kExrInvalidData;
            const int ci = add_chunk(o + 8, dlen, (int)W, (int)nl);
            if (ci < 0) return kExrInvalidData;
            // rows it writes: ZIP / RLE from line_no, NONE from the block index (:4151-4168)
            const int64_t row0 = comp == 0 ? (int64_t)y : lno;
            for (int64_t v = 0; v < nl; ++v) {
                const int64_t row = line_order == 0 ? row0 + v : H - 1 - (row0 + v);
                if (row < 0 || row >= H) return kExrInvalidData;  // (tinyexr writes outside its image)
                P.map[(size_t)row] = make_int2(ci, (int)v);
            }
        }
    }
    // RGBA channel choice (:6686-6703, :6706, :6766-6783): the last channel of each name
    for (int k = 0; k < 4; ++k) P.src[k] = -1;
    for (int c = 0; c < P.nch; ++c) {
        const std::string& n = chans[(size_t)c].name;
        if (n == "R") P.src[0] = c;
        else if (n == "G") P.src[1] = c;
        else if (n == "B") P.src[2] = c;
        else if (n == "A") P.src[3] = c;
    }
    if (P.nch == 1) {
        for (int k = 0; k < 4; ++k) P.src[k] = 0;
    } else if (P.src[0] < 0 || P.src[1] < 0 || P.src[2] < 0) {
        return kExrInvalidData;
    }
    return kExrOk;
}

// Byte p of a chunk's decoded pixel data (the even / odd reorder: p even -> t[p/2], odd ->
// t[(m+1)/2 + p/2]; bytes past what the decompressor produced are 0).
ICX_HD uint32_t exr_byte(const uint8_t* file, const uint8_t* scratch, const ExrChunk& c, int64_t p) {
    if (c.mode == 0) return file[c.src + p];
    const int64_t m = c.produced;
    if (p >= m) return 0;
    const uint8_t* t = scratch + c.scratch;
    if (c.mode == 3) return t[p];  // PIZ: the pixel bytes in order (no predictor or reorder)
    return (p & 1) ? t[(m + 1) / 2 + (p >> 1)] : t[p >> 1];
}

struct ExrConv {
    int w, h, nch, pds, tiled, tx, ty, ntx, line_order;
    int src[4];
};

// Output pixel px (RGBA bits) as LoadEXRFromMemory's loops assemble it (:6706-6860).
ICX_HD uint4 exr_pixel(const uint8_t* file, const uint8_t* scratch, const ExrChunk* ch, const int2* map,
                       const int32_t* tile_h, const int32_t* ctype, const int32_t* coffs, const ExrConv& cv, int64_t px) {
    const int x = (int)(px % cv.w), y = (int)(px / cv.w);
    int ci = -1;
    int64_t v = 0, u = x;
    if (cv.tiled) {
        const int tcx = x / cv.tx, tcy = y / cv.ty;
        ci = map[(int64_t)tcy * cv.ntx + tcx].x;
        u = x - (int64_t)tcx * cv.tx;
        const int j = y - tcy * cv.ty;
        v = cv.line_order == 0 ? j : cv.ty - 1 - j;  // DecodePixelData's row for tiles (height = tile_size_y)
        if (ci >= 0 && v >= tile_h[ci]) ci = -1;     // (a row that tile did not write)
    } else {
        const int2 e = map[y];
        ci = e.x;
        v = e.y;
    }
    uint32_t o[4] = {0, 0, 0, 0};
    if (ci >= 0) {
        const ExrChunk c = ch[ci];
        const int64_t wc = c.width;
        for (int k = 0; k < 4; ++k) {
            const int s = cv.src[k];
            if (s < 0) {
                o[k] = 0x3f800000u;  // no A: 1.0 (:6825, :6845)
                continue;
            }
            const int ty = ctype[s];
            const int64_t pb = v * cv.pds * wc + (int64_t)coffs[s] * wc + u * (ty == 1 ? 2 : 4);
            if (ty == 1) {
                o[k] = exr_half_bits(exr_byte(file, scratch, c, pb) | (exr_byte(file, scratch, c, pb + 1) << 8));
            } else {
                o[k] = exr_byte(file, scratch, c, pb) | (exr_byte(file, scratch, c, pb + 1) << 8) |
                       (exr_byte(file, scratch, c, pb + 2) << 16) | (exr_byte(file, scratch, c, pb + 3) << 24);
            }
        }
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

}  // namespace icx
