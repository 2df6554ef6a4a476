// jpeg.hip — JPEG decode for the embedding path: Huffman on the host, pixel
// reconstruction on the GPU.  Replaces the PIL decode of embedding/main.py:97
// (Image.open(BytesIO(bytes)).convert("RGB")) for baseline JPEGs, bit-exact with
// Pillow 12.2 / libjpeg-turbo 3.1 default decompression (JDCT_ISLOW, fancy
// upsampling, JCS_YCbCr -> JCS_RGB); SURVEY.md §8(f) rank 4.
//
// Host (per image, one thread per image of a batch): marker parse (DQT, SOF0/1,
// DHT, DRI, SOS, APP0/APP14 colour-space rules of jdapimin.c), Huffman decode of
// the single interleaved scan into quantised coefficients (natural order, int16,
// one 8x8 block = 128 B), restart markers.  Everything else — progressive or
// arithmetic coding, 12-bit samples, multi-scan sequential files, CMYK/YCCK/RGB
// colour spaces, sampling ratios other than 1 and 2 — is reported as
// unsupported (rc_jpeg_info.supported = 0) and the caller decodes on the host
// with PIL, exactly as the reference does.
// Device: jpeg_idct_kernel (8 lanes per block: dequantise, jidctint.c "islow"
// column then row pass, descale, clamp to [0,255] as libjpeg-turbo's SIMD
// islow does) writes 8x8 u8 sample blocks; jpeg_color_kernel (one lane per
// output pixel) applies jdsample.c's fancy upsampling (h2v1, h1v2, h2v2
// triangle filters with replicated edge rows/columns, plain replication when the
// downsampled width is <= 2) and jdcolor.c's fixed-point YCbCr -> RGB, writing
// HWC u8 RGB straight into the caller's buffer (the input of rc_embed's resize).
// rc_jpeg_decode_resized fuses the colour pass with Pillow's horizontal resample
// (jpeg_color_resize_h_kernel: a source row's RGB built in LDS, each output pixel
// filtered from it) and runs the vertical pass per image (jpeg_resize_v_kernel):
// the full-size RGB image is never written, and the result equals PIL decode +
// Image.resize (ViTImageProcessor's resize, embedding/main.py:97,107) bit for bit.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include <map>
#include <tuple>
#include <type_traits>

#include "rc_common.h"
#include "resample.h"

namespace rc {
namespace jpeg {

static const uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct Huff {
    bool present = false;
    // canonical decoding: maxcode[l] (codes of length l are < maxcode[l]),
    // valptr[l] - mincode[l] indexes vals; a 9-bit lookahead table for speed
    int32_t maxcode[18];
    int32_t delta[17];
    uint8_t vals[256];
    uint16_t look[512];  // (length << 8) | value, length 0 = not in table
};

struct Comp {
    int id = 0, h = 1, v = 1, tq = 0, td = 0, ta = 0;
    int bw = 0, bh = 0;  // blocks per plane (MCU padded)
    int64_t blk0 = 0;    // first block of the plane within the image
};

struct Header {
    int width = 0, height = 0, ncomp = 0, hmax = 1, vmax = 1, restart = 0, mcux = 0, mcuy = 0;
    Comp c[3];
    uint16_t qt[4][64];
    bool qt_present[4] = {false, false, false, false};
    Huff dc[4], ac[4];
    const uint8_t *scan = nullptr;
    const uint8_t *end = nullptr;
    int scan_ncomp = 0, scan_comp[3] = {0, 0, 0};
    bool jfif = false, adobe = false;
    int adobe_transform = -1;
    int64_t blocks = 0;
    bool supported = false;
    std::string why;
};

static void build_huff(Huff &t, const uint8_t *counts, const uint8_t *vals, int nvals) {
    t.present = true;
    std::memcpy(t.vals, vals, nvals);
    int code = 0, k = 0;
    std::memset(t.look, 0, sizeof(t.look));
    for (int l = 1; l <= 16; ++l) {
        t.delta[l] = k - code;  // index of code c of length l = c + delta[l]
        for (int i = 0; i < counts[l - 1]; ++i, ++k, ++code) {
            if (l <= 9) {
                const int shift = 9 - l;
                for (int f = 0; f < (1 << shift); ++f) t.look[(code << shift) | f] = (uint16_t)((l << 8) | vals[k]);
            }
        }
        t.maxcode[l] = code;  // exclusive
        code <<= 1;
    }
    t.maxcode[17] = 0x7fffffff;
}

static inline int u16be(const uint8_t *p) { return (p[0] << 8) | p[1]; }

// Marker walk up to the first SOS.  Returns false (with why) when the stream is
// not one this decoder reconstructs; hard format errors throw.
static void parse(const uint8_t *data, int64_t len, Header &hd) {
    const uint8_t *p = data, *end = data + len;
    RC_REQUIRE(len >= 4 && p[0] == 0xFF && p[1] == 0xD8, RC_ERR_INVALID, "not a JPEG stream (no SOI)");
    p += 2;
    bool sof = false;
    auto unsupported = [&](const std::string &w) {
        hd.supported = false;
        hd.why = w;
    };
    hd.supported = true;
    while (true) {
        while (p < end && *p != 0xFF) ++p;  // tolerate garbage between markers (libjpeg warns)
        while (p < end && *p == 0xFF) ++p;
        RC_REQUIRE(p < end, RC_ERR_INVALID, "JPEG: no SOS before end of data");
        const int m = *p++;
        if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
        if (m == 0xD9) throw Error(RC_ERR_INVALID, "JPEG: EOI before SOS");
        RC_REQUIRE(end - p >= 2, RC_ERR_INVALID, "JPEG: truncated marker");
        const int L = u16be(p);
        RC_REQUIRE(L >= 2 && end - p >= L, RC_ERR_INVALID, "JPEG: truncated marker segment");
        const uint8_t *s = p + 2, *se = p + L;
        p += L;
        if (m == 0xDB) {  // DQT
            while (s < se) {
                const int pq = s[0] >> 4, tq = s[0] & 15;
                RC_REQUIRE(tq < 4 && pq < 2, RC_ERR_INVALID, "JPEG: bad DQT");
                ++s;
                RC_REQUIRE(se - s >= (pq ? 128 : 64), RC_ERR_INVALID, "JPEG: short DQT");
                for (int k = 0; k < 64; ++k) {
                    const int v = pq ? u16be(s + 2 * k) : s[k];
                    hd.qt[tq][kZigzag[k]] = (uint16_t)v;
                }
                s += pq ? 128 : 64;
                hd.qt_present[tq] = true;
            }
        } else if (m == 0xC4) {  // DHT
            while (s < se) {
                RC_REQUIRE(se - s >= 17, RC_ERR_INVALID, "JPEG: short DHT");
                const int tc = s[0] >> 4, th = s[0] & 15;
                RC_REQUIRE(tc < 2 && th < 4, RC_ERR_INVALID, "JPEG: bad DHT");
                int n = 0;
                for (int i = 1; i <= 16; ++i) n += s[i];
                RC_REQUIRE(n <= 256 && se - s >= 17 + n, RC_ERR_INVALID, "JPEG: bad DHT counts");
                build_huff(tc ? hd.ac[th] : hd.dc[th], s + 1, s + 17, n);
                s += 17 + n;
            }
        } else if (m >= 0xC0 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {  // SOFn
            RC_REQUIRE(se - s >= 6, RC_ERR_INVALID, "JPEG: short SOF");
            if (m != 0xC0 && m != 0xC1) unsupported("SOF" + std::to_string(m - 0xC0) + " (progressive / lossless / arithmetic)");
            if (s[0] != 8) unsupported("sample precision " + std::to_string(s[0]));
            hd.height = u16be(s + 1);
            hd.width = u16be(s + 3);
            hd.ncomp = s[5];
            RC_REQUIRE(se - s >= 6 + 3 * hd.ncomp, RC_ERR_INVALID, "JPEG: short SOF");
            if (hd.ncomp != 1 && hd.ncomp != 3) {
                unsupported(std::to_string(hd.ncomp) + " components");
                hd.ncomp = std::min(hd.ncomp, 3);
            }
            for (int i = 0; i < hd.ncomp; ++i) {
                hd.c[i].id = s[6 + 3 * i];
                hd.c[i].h = s[7 + 3 * i] >> 4;
                hd.c[i].v = s[7 + 3 * i] & 15;
                hd.c[i].tq = s[8 + 3 * i] & 3;
                RC_REQUIRE(hd.c[i].h >= 1 && hd.c[i].h <= 4 && hd.c[i].v >= 1 && hd.c[i].v <= 4, RC_ERR_INVALID,
                           "JPEG: bad sampling factor");
            }
            sof = true;
        } else if (m == 0xCC) {
            unsupported("arithmetic coding");
        } else if (m == 0xDD) {  // DRI
            RC_REQUIRE(se - s >= 2, RC_ERR_INVALID, "JPEG: short DRI");
            hd.restart = u16be(s);
        } else if (m == 0xE0) {
            if (se - s >= 5 && std::memcmp(s, "JFIF\0", 5) == 0) hd.jfif = true;
        } else if (m == 0xEE) {
            if (se - s >= 12 && std::memcmp(s, "Adobe", 5) == 0) {
                hd.adobe = true;
                hd.adobe_transform = s[11];
            }
        } else if (m == 0xDA) {  // SOS
            RC_REQUIRE(sof, RC_ERR_INVALID, "JPEG: SOS before SOF");
            RC_REQUIRE(se - s >= 1, RC_ERR_INVALID, "JPEG: short SOS");
            hd.scan_ncomp = s[0];
            RC_REQUIRE(hd.scan_ncomp >= 1 && hd.scan_ncomp <= 4 && se - s >= 4 + 2 * hd.scan_ncomp, RC_ERR_INVALID,
                       "JPEG: bad SOS");
            for (int i = 0; i < std::min(hd.scan_ncomp, 3); ++i) {
                const int cid = s[1 + 2 * i];
                int ci = -1;
                for (int j = 0; j < hd.ncomp; ++j)
                    if (hd.c[j].id == cid) ci = j;
                RC_REQUIRE(ci >= 0, RC_ERR_INVALID, "JPEG: SOS names an unknown component");
                hd.scan_comp[i] = ci;
                hd.c[ci].td = s[2 + 2 * i] >> 4;
                hd.c[ci].ta = s[2 + 2 * i] & 15;
            }
            const uint8_t *t = s + 1 + 2 * hd.scan_ncomp;
            if (t[0] != 0 || t[1] != 63 || t[2] != 0) unsupported("spectral selection / successive approximation");
            if (hd.scan_ncomp != hd.ncomp) unsupported("multi-scan sequential JPEG");
            hd.scan = p;
            hd.end = end;
            break;
        }
    }
    if (!hd.supported) return;
    RC_REQUIRE(hd.width > 0, RC_ERR_INVALID, "JPEG: zero width");
    if (hd.height == 0) return unsupported("DNL-defined height");
    // colour space as jdapimin.c default_decompress_parms: 3 components are
    // YCbCr unless an Adobe marker says transform 0 or (without JFIF/Adobe)
    // the component ids spell R, G, B
    if (hd.ncomp == 3) {
        bool rgb = false;
        if (hd.adobe) rgb = hd.adobe_transform == 0;
        else if (!hd.jfif) rgb = hd.c[0].id == 82 && hd.c[1].id == 71 && hd.c[2].id == 66;
        if (rgb) return unsupported("RGB colour space");
    }
    hd.hmax = hd.vmax = 1;
    for (int i = 0; i < hd.ncomp; ++i) {
        hd.hmax = std::max(hd.hmax, hd.c[i].h);
        hd.vmax = std::max(hd.vmax, hd.c[i].v);
    }
    for (int i = 0; i < hd.ncomp; ++i) {
        const int rx = hd.hmax / hd.c[i].h, ry = hd.vmax / hd.c[i].v;
        if (hd.hmax % hd.c[i].h || hd.vmax % hd.c[i].v || rx > 2 || ry > 2)
            return unsupported("sampling ratio other than 1 or 2");
        if (!hd.qt_present[hd.c[i].tq]) throw Error(RC_ERR_INVALID, "JPEG: missing quantisation table");
        if (!hd.dc[hd.c[i].td].present || !hd.ac[hd.c[i].ta].present)
            throw Error(RC_ERR_INVALID, "JPEG: missing Huffman table");
    }
    if (hd.ncomp == 1) {  // non-interleaved: MCU = one block, sampling factors ignored
        hd.hmax = hd.vmax = 1;
        hd.c[0].h = hd.c[0].v = 1;
    }
    hd.mcux = (hd.width + 8 * hd.hmax - 1) / (8 * hd.hmax);
    hd.mcuy = (hd.height + 8 * hd.vmax - 1) / (8 * hd.vmax);
    int64_t b = 0;
    for (int i = 0; i < hd.ncomp; ++i) {
        hd.c[i].bw = hd.mcux * hd.c[i].h;
        hd.c[i].bh = hd.mcuy * hd.c[i].v;
        hd.c[i].blk0 = b;
        b += (int64_t)hd.c[i].bw * hd.c[i].bh;
    }
    hd.blocks = b;
}

// Entropy-coded segment reader: byte unstuffing; at a marker (or the end of
// the buffer) it feeds zero bits and counts them, so a decoder that consumes
// any of them has run past the segment (a damaged or truncated stream: an
// error here, never silently zero-filled).
struct Bits {
    const uint8_t *p, *end;
    uint64_t acc = 0;
    int n = 0, fake = 0;
    bool hit_marker = false;
    int marker = 0;
    void fill() {
        while (n <= 56) {
            int b = 0;
            if (!hit_marker && p < end) {
                b = *p;
                if (b == 0xFF) {
                    const int nx = p + 1 < end ? p[1] : -1;
                    if (nx == 0x00) {
                        p += 2;
                    } else {  // a marker: p stays on its 0xFF
                        hit_marker = true;
                        marker = nx < 0 ? 0 : nx;
                        b = 0;
                        fake += 8;
                    }
                } else {
                    ++p;
                }
            } else {
                hit_marker = true;
                fake += 8;
            }
            acc |= (uint64_t)b << (56 - n);
            n += 8;
        }
    }
    inline int peek(int k) {
        if (n < k) fill();
        return (int)(acc >> (64 - k));
    }
    inline void skip(int k) {
        acc <<= k;
        n -= k;
    }
    inline int get(int k) {
        if (k == 0) return 0;
        const int v = peek(k);
        skip(k);
        return v;
    }
    bool overrun() const { return fake > n; }
    // byte-align and step over the expected RSTn marker
    void restart(int rst) {
        const bool at_marker = hit_marker ? marker == rst : (p + 1 < end && p[0] == 0xFF && p[1] == rst);
        RC_REQUIRE(at_marker, RC_ERR_INVALID, "JPEG: missing restart marker");
        p += 2;
        acc = 0;
        n = fake = 0;
        hit_marker = false;
        marker = 0;
    }
};

static inline int decode_sym(Bits &b, const Huff &t) {
    const int l9 = b.peek(9);
    const uint16_t e = t.look[l9];
    if (e) {
        b.skip(e >> 8);
        return e & 0xFF;
    }
    int code = b.peek(16);
    for (int l = 10; l <= 16; ++l) {
        const int c = code >> (16 - l);
        if (c < t.maxcode[l]) {
            b.skip(l);
            const int idx = c + t.delta[l];
            if (idx < 0 || idx > 255) throw Error(RC_ERR_INVALID, "JPEG: corrupt Huffman data");
            return t.vals[idx];
        }
    }
    throw Error(RC_ERR_INVALID, "JPEG: corrupt Huffman data");
}

static inline int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

static void decode_block(Bits &b, const Huff &dc, const Huff &ac, int &pred, int16_t *blk) {
    int s = decode_sym(b, dc);
    if (s) {
        RC_REQUIRE(s <= 11, RC_ERR_INVALID, "JPEG: corrupt DC");
        pred += extend(b.get(s), s);
    }
    blk[0] = (int16_t)pred;
    for (int k = 1; k < 64; ++k) {
        const int rs = decode_sym(b, ac);
        const int r = rs >> 4;
        s = rs & 15;
        if (s) {
            k += r;
            RC_REQUIRE(k < 64, RC_ERR_INVALID, "JPEG: corrupt AC run");
            blk[kZigzag[k]] = (int16_t)extend(b.get(s), s);
        } else {
            if (r != 15) break;
            k += 15;
        }
    }
}

// Quantised coefficients of every block (natural order), planes in component order.
static void decode_coefficients(const Header &hd, int16_t *coef) {
    std::memset(coef, 0, (size_t)hd.blocks * 64 * sizeof(int16_t));
    Bits b{hd.scan, hd.end};
    int pred[3] = {0, 0, 0};
    const int64_t nmcu = hd.ncomp == 1 ? (int64_t)((hd.width + 7) / 8) * ((hd.height + 7) / 8)
                                       : (int64_t)hd.mcux * hd.mcuy;
    const int bw1 = (hd.width + 7) / 8;  // non-interleaved raster width
    int expect_rst = 0;
    for (int64_t mcu = 0; mcu < nmcu; ++mcu) {
        if (hd.restart && mcu > 0 && mcu % hd.restart == 0) {
            b.restart(0xD0 + expect_rst);
            expect_rst = (expect_rst + 1) & 7;
            pred[0] = pred[1] = pred[2] = 0;
        }
        if (hd.ncomp == 1) {
            const int by = (int)(mcu / bw1), bx = (int)(mcu % bw1);
            const Comp &c = hd.c[0];
            decode_block(b, hd.dc[c.td], hd.ac[c.ta], pred[0], coef + (c.blk0 + (int64_t)by * c.bw + bx) * 64);
        } else {
            const int my = (int)(mcu / hd.mcux), mx = (int)(mcu % hd.mcux);
            for (int si = 0; si < hd.scan_ncomp; ++si) {
                const int ci = hd.scan_comp[si];
                const Comp &c = hd.c[ci];
                for (int v = 0; v < c.v; ++v)
                    for (int h = 0; h < c.h; ++h) {
                        const int64_t blk = c.blk0 + (int64_t)(my * c.v + v) * c.bw + (mx * c.h + h);
                        decode_block(b, hd.dc[c.td], hd.ac[c.ta], pred[ci], coef + blk * 64);
                    }
            }
        }
        RC_REQUIRE(!b.overrun(), RC_ERR_INVALID, "JPEG: premature end of entropy-coded data");
    }
}

static void fill_info(const Header &hd, rc_jpeg_info *info) {
    std::memset(info, 0, sizeof(*info));
    info->width = hd.width;
    info->height = hd.height;
    info->ncomp = hd.ncomp;
    info->supported = hd.supported ? 1 : 0;
    if (!hd.supported) return;
    info->hmax = hd.hmax;
    info->vmax = hd.vmax;
    info->restart_interval = hd.restart;
    info->mcux = hd.mcux;
    info->mcuy = hd.mcuy;
    for (int i = 0; i < hd.ncomp; ++i) {
        info->h[i] = hd.c[i].h;
        info->v[i] = hd.c[i].v;
        info->bw[i] = hd.c[i].bw;
        info->bh[i] = hd.c[i].bh;
    }
    info->blocks = hd.blocks;
}

// ------------------------------------------------------------------ device --
// Per-image reconstruction descriptor (device memory).
struct Desc {
    int32_t W, H, ncomp, pad;
    int32_t rx[3], ry[3];  // upsampling ratio per component (1 or 2)
    int32_t dw[3], dh[3];  // downsampled (real) component size in samples
    int32_t bw[3], pad2;
    int64_t blk0[3];       // global block index of each plane
    int64_t rgb_off;       // byte offset of the HWC RGB output
};

constexpr int FIX_0_298631336 = 2446, FIX_0_390180644 = 3196, FIX_0_541196100 = 4433, FIX_0_765366865 = 6270,
              FIX_0_899976223 = 7373, FIX_1_175875602 = 9633, FIX_1_501321110 = 12299, FIX_1_847759065 = 15137,
              FIX_1_961570560 = 16069, FIX_2_053119869 = 16819, FIX_2_562915447 = 20995, FIX_3_072711026 = 25172;

// One 8-point islow IDCT (jidctint.c) on in[0..7] (already dequantised / pass-1
// scaled); returns the 8 undescaled outputs in o[] (descale by the caller).
__device__ __forceinline__ void idct8(const int *in, int *o) {
    int z2 = in[2], z3 = in[6];
    int z1 = (z2 + z3) * FIX_0_541196100;
    const int tmp2e = z1 + z3 * (-FIX_1_847759065);
    const int tmp3e = z1 + z2 * FIX_0_765366865;
    z2 = in[0];
    z3 = in[4];
    const int tmp0e = (z2 + z3) * (1 << 13);
    const int tmp1e = (z2 - z3) * (1 << 13);
    const int tmp10 = tmp0e + tmp3e, tmp13 = tmp0e - tmp3e, tmp11 = tmp1e + tmp2e, tmp12 = tmp1e - tmp2e;
    int tmp0 = in[7], tmp1 = in[5], tmp2 = in[3], tmp3 = in[1];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    int z4 = tmp1 + tmp3;
    const int z5 = (z3 + z4) * FIX_1_175875602;
    tmp0 *= FIX_0_298631336;
    tmp1 *= FIX_2_053119869;
    tmp2 *= FIX_3_072711026;
    tmp3 *= FIX_1_501321110;
    z1 *= -FIX_0_899976223;
    z2 *= -FIX_2_562915447;
    z3 *= -FIX_1_961570560;
    z4 *= -FIX_0_390180644;
    z3 += z5;
    z4 += z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    o[0] = tmp10 + tmp3;
    o[7] = tmp10 - tmp3;
    o[1] = tmp11 + tmp2;
    o[6] = tmp11 - tmp2;
    o[2] = tmp12 + tmp1;
    o[5] = tmp12 - tmp1;
    o[3] = tmp13 + tmp0;
    o[4] = tmp13 - tmp0;
}

__device__ __forceinline__ int descale(int x, int n) { return (x + (1 << (n - 1))) >> n; }

// 64 lanes = 8 blocks; lane (blk, r): loads coefficient row r, does column r in
// pass 1 and row r in pass 2 (exchange through LDS), stores 8 samples.
__global__ __launch_bounds__(64) void jpeg_idct_kernel(const int16_t *__restrict__ coef, const int32_t *__restrict__ qsel,
                                                      const uint16_t *__restrict__ qtab, int64_t nblocks,
                                                      uint8_t *__restrict__ planes) {
    __shared__ int ws[8][8][9];  // [block][row][col], padded
    const int lane = threadIdx.x, lb = lane >> 3, r = lane & 7;
    const int64_t blk = (int64_t)blockIdx.x * 8 + lb;
    const bool valid = blk < nblocks;
    if (valid) {
        const uint16_t *q = qtab + (int64_t)qsel[blk] * 64 + r * 8;
        const int4 raw = *reinterpret_cast<const int4 *>(coef + blk * 64 + r * 8);
        const int16_t *c = reinterpret_cast<const int16_t *>(&raw);
#pragma unroll
        for (int k = 0; k < 8; ++k) ws[lb][r][k] = (int)c[k] * (int)q[k];
    }
    __syncthreads();
    int in[8], o[8];
    // pass 1: column r -> work values scaled by 2^PASS1_BITS (descale CONST_BITS - PASS1_BITS = 11)
#pragma unroll
    for (int k = 0; k < 8; ++k) in[k] = ws[lb][k][r];
    idct8(in, o);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) ws[lb][k][r] = descale(o[k], 11);
    __syncthreads();
    // pass 2: row r, descale CONST_BITS + PASS1_BITS + 3 = 18, +128, clamp
#pragma unroll
    for (int k = 0; k < 8; ++k) in[k] = ws[lb][r][k];
    idct8(in, o);
    if (!valid) return;
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int v = min(max(descale(o[k], 18) + 128, 0), 255);
        if (k < 4) lo |= (uint32_t)v << (8 * k);
        else hi |= (uint32_t)v << (8 * (k - 4));
    }
    *reinterpret_cast<uint2 *>(planes + blk * 64 + r * 8) = make_uint2(lo, hi);
}

__device__ __forceinline__ int sample_at(const uint8_t *__restrict__ planes, const Desc &d, int c, int x, int y) {
    const int64_t blk = d.blk0[c] + (int64_t)(y >> 3) * d.bw[c] + (x >> 3);
    return planes[blk * 64 + (y & 7) * 8 + (x & 7)];
}

// Component c's sample at output pixel (x, y) through jdsample.c's upsampler; at(c, x, y) reads
// one stored sample (from the planes in HBM, or from a band's copy of them in LDS).
template <typename At>
__device__ __forceinline__ int upsampled_t(const Desc &d, int c, int x, int y, At &&at) {
    const int rx = d.rx[c], ry = d.ry[c];
    if (rx == 1 && ry == 1) return at(c, x, y);
    const int dw = d.dw[c], dh = d.dh[c];
    if (ry == 1) {  // h2v1
        const int i = x >> 1;
        const int s = at(c, i, y);
        if (dw <= 2) return s;
        if ((x & 1) == 0) return i == 0 ? s : (3 * s + at(c, i - 1, y) + 1) >> 2;
        return i == dw - 1 ? s : (3 * s + at(c, i + 1, y) + 2) >> 2;
    }
    const int j = y >> 1, vv = y & 1;
    const int far = vv == 0 ? max(j - 1, 0) : min(j + 1, dh - 1);
    if (rx == 1) {  // h1v2 (always fancy)
        return (3 * at(c, x, j) + at(c, x, far) + (vv == 0 ? 1 : 2)) >> 2;
    }
    // h2v2
    const int i = x >> 1;
    if (dw <= 2) return at(c, i, j);
    auto colsum = [&](int ii) { return 3 * at(c, ii, j) + at(c, ii, far); };
    const int cs = colsum(i);
    if ((x & 1) == 0) return i == 0 ? (cs * 4 + 8) >> 4 : (3 * cs + colsum(i - 1) + 8) >> 4;
    return i == dw - 1 ? (cs * 4 + 7) >> 4 : (3 * cs + colsum(i + 1) + 7) >> 4;
}

__device__ __forceinline__ int upsampled(const uint8_t *__restrict__ planes, const Desc &d, int c, int x, int y) {
    return upsampled_t(d, c, x, y, [&](int cc, int xx, int yy) { return sample_at(planes, d, cc, xx, yy); });
}

// The 8-row block rows of component c that the upsampler reads for the image rows [y_lo, y_hi):
// [*br0, *br0 + *nbr).  A v2 component also reads the chroma row beyond each end (jdsample.c's
// "far" row, clamped to the plane).  Host and device compute it alike (the band kernel's LDS plan).
__host__ __device__ __forceinline__ void plane_block_rows(const Desc &d, int c, int y_lo, int y_hi, int *br0, int *nbr) {
    int r_lo = y_lo, r_hi = y_hi - 1;
    if (d.ry[c] == 2) {
        r_lo = (y_lo >> 1) - 1;
        r_lo = r_lo < 0 ? 0 : r_lo;
        r_hi = ((y_hi - 1) >> 1) + 1;
        r_hi = r_hi > d.dh[c] - 1 ? d.dh[c] - 1 : r_hi;
    }
    *br0 = r_lo >> 3;
    *nbr = (r_hi >> 3) - *br0 + 1;
}

// grid (ceil(max_pixels / 256), n): one lane per output pixel of image blockIdx.y.
__global__ __launch_bounds__(256) void jpeg_color_kernel(const uint8_t *__restrict__ planes, const Desc *__restrict__ descs,
                                                        uint8_t *__restrict__ rgb) {
    const Desc d = descs[blockIdx.y];
    // W*H < 2^31 (checked at decode): 32-bit index math, no emulated 64-bit divide
    const int p = (int)blockIdx.x * 256 + (int)threadIdx.x;
    if (p >= d.W * d.H) return;
    const int y = p / d.W, x = p - y * d.W;
    uint8_t *o = rgb + d.rgb_off + (int64_t)p * 3;
    const int Y = upsampled(planes, d, 0, x, y);
    if (d.ncomp == 1) {
        o[0] = o[1] = o[2] = (uint8_t)Y;
        return;
    }
    const int cb = upsampled(planes, d, 1, x, y) - 128, cr = upsampled(planes, d, 2, x, y) - 128;
    // jdcolor.c build_ycc_rgb_table / ycc_rgb_convert (SCALEBITS 16)
    const int R = Y + ((__mul24(91881, cr) + 32768) >> 16);
    const int G = Y + ((__mul24(-22554, cb) + 32768 - __mul24(46802, cr)) >> 16);
    const int B = Y + ((__mul24(116130, cb) + 32768) >> 16);
    o[0] = (uint8_t)min(max(R, 0), 255);
    o[1] = (uint8_t)min(max(G, 0), 255);
    o[2] = (uint8_t)min(max(B, 0), 255);
}

// Per-image plan of the fused decode → resize (rc_jpeg_decode_resized), Pillow's
// ImagingResample order: horizontal pass over the source rows the vertical pass reads
// ([y0, y0 + Hs)), into tmp [Hs][S][3], then the vertical pass into out [S][S][3]; an
// axis whose size already is S is skipped (need_h / need_v), as Pillow skips it.
struct RDesc {
    int32_t S, need_h, need_v, y0, Hs, hk, vk, bh;  // bh: output rows per block of the band kernel
    const int *hb, *hc;  // horizontal bounds [S][2] (xmin, count) / coefficients [S][hk]
    const int *vb, *vc;  // vertical bounds relative to y0 / coefficients [S][vk]
    int64_t tmp_off, out_off;
};

__device__ __forceinline__ uint8_t clip8_22(int acc) {
    const int v = acc >> 22;
    return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

__device__ __forceinline__ void ycc_rgb(const uint8_t *__restrict__ planes, const Desc &d, int x, int y, int &R, int &G,
                                        int &B) {
    const int Y = upsampled(planes, d, 0, x, y);
    if (d.ncomp == 1) {
        R = G = B = Y;
        return;
    }
    const int cb = upsampled(planes, d, 1, x, y) - 128, cr = upsampled(planes, d, 2, x, y) - 128;
    R = min(max(Y + ((__mul24(91881, cr) + 32768) >> 16), 0), 255);
    G = min(max(Y + ((__mul24(-22554, cb) + 32768 - __mul24(46802, cr)) >> 16), 0), 255);
    B = min(max(Y + ((__mul24(116130, cb) + 32768) >> 16), 0), 255);
}

constexpr int RS_WIN = 16384;  // source pixels of one row staged in LDS at a time (48 KB)

// grid (max rows, n), 256 lanes: block (y, i) produces row y of image i's horizontal pass
// (or, without one, its colour row).  The source row's RGB is built in LDS over windows
// of RS_WIN pixels; every output pixel whose taps lie inside the window is filtered from
// it (Pillow's fixed-point sum, 22 fractional bits, rounding 1 << 21, clip).
__global__ __launch_bounds__(256) void jpeg_color_resize_h_kernel(const uint8_t *__restrict__ planes,
                                                                 const Desc *__restrict__ descs,
                                                                 const RDesc *__restrict__ rdescs, uint8_t *__restrict__ tmp,
                                                                 uint8_t *__restrict__ out) {
    __shared__ uint8_t row[RS_WIN * 3];
    __shared__ int span[2];  // [1]: the end of the current window's outputs
    const Desc d = descs[blockIdx.y];
    const RDesc r = rdescs[blockIdx.y];
    const int y = blockIdx.x;
    if (y >= r.Hs) return;  // block-uniform
    const int sy = r.y0 + y, S = r.S;
    uint8_t *dst = (r.need_v ? tmp + r.tmp_off : out + r.out_off) + (int64_t)y * S * 3;
    if (!r.need_h) {  // width already S: the colour row as it is
        for (int x = threadIdx.x; x < d.W; x += 256) {
            int R, G, B;
            ycc_rgb(planes, d, x, sy, R, G, B);
            dst[3 * x] = (uint8_t)R;
            dst[3 * x + 1] = (uint8_t)G;
            dst[3 * x + 2] = (uint8_t)B;
        }
        return;
    }
    for (int xo0 = 0; xo0 < S;) {
        // outputs [xo0, xo1) whose taps fit one window starting at xmin(xo0): the first output
        // past it, found by every lane testing its outputs at once (a min over the block);
        // a row of <= RS_WIN pixels is one window
        const int w0 = r.hb[2 * xo0];
        int xo1 = S;
        if (d.W - w0 > RS_WIN) {
            if (threadIdx.x == 0) span[1] = S;
            __syncthreads();
            for (int xo = xo0 + 1 + (int)threadIdx.x; xo < S; xo += 256)
                if (r.hb[2 * xo] + r.hb[2 * xo + 1] > w0 + RS_WIN) atomicMin(&span[1], xo);
            __syncthreads();
            xo1 = span[1];
        }
        const int w1 = min(d.W, w0 + RS_WIN);
        for (int x = w0 + (int)threadIdx.x; x < w1; x += 256) {
            int R, G, B;
            ycc_rgb(planes, d, x, sy, R, G, B);
            row[3 * (x - w0)] = (uint8_t)R;
            row[3 * (x - w0) + 1] = (uint8_t)G;
            row[3 * (x - w0) + 2] = (uint8_t)B;
        }
        __syncthreads();
        for (int xo = xo0 + (int)threadIdx.x; xo < xo1; xo += 256) {
            const int xmin = r.hb[2 * xo] - w0, xn = r.hb[2 * xo + 1];
            const int *c = r.hc + xo * r.hk;
            int a0 = 1 << 21, a1 = 1 << 21, a2 = 1 << 21;
            for (int k = 0; k < xn; ++k) {
                const uint8_t *p = row + 3 * (xmin + k);
                a0 = resample_tap(a0, p[0], c[k]);
                a1 = resample_tap(a1, p[1], c[k]);
                a2 = resample_tap(a2, p[2], c[k]);
            }
            dst[3 * xo] = clip8_22(a0);
            dst[3 * xo + 1] = clip8_22(a1);
            dst[3 * xo + 2] = clip8_22(a2);
        }
        __syncthreads();  // the window is rebuilt next
        xo0 = xo1;
    }
}

// grid (ceil(S*S / 256), n): Pillow's vertical pass of image blockIdx.y (need_v only).
__global__ __launch_bounds__(256) void jpeg_resize_v_kernel(const RDesc *__restrict__ rdescs,
                                                           const uint8_t *__restrict__ tmp, uint8_t *__restrict__ out) {
    const RDesc r = rdescs[blockIdx.y];
    if (!r.need_v) return;
    const int S = r.S;
    const int p = (int)blockIdx.x * 256 + (int)threadIdx.x;
    if (p >= S * S) return;
    const int yo = p / S, x = p - yo * S;
    const int ymin = r.vb[2 * yo], yn = r.vb[2 * yo + 1];
    const int *c = r.vc + yo * r.vk;
    const uint8_t *col = tmp + r.tmp_off + ((int64_t)ymin * S + x) * 3;
    int a0 = 1 << 21, a1 = 1 << 21, a2 = 1 << 21;
    for (int k = 0; k < yn; ++k) {
        const uint8_t *q = col + (int64_t)k * S * 3;
        a0 = resample_tap(a0, q[0], c[k]);
        a1 = resample_tap(a1, q[1], c[k]);
        a2 = resample_tap(a2, q[2], c[k]);
    }
    uint8_t *o = out + r.out_off + (int64_t)p * 3;
    o[0] = clip8_22(a0);
    o[1] = clip8_22(a1);
    o[2] = clip8_22(a2);
}


// Band-fused decode → resize (rc_jpeg_decode_resized when every image's band fits in LDS):
// grid (max bands, n), 256 lanes = 4 waves; block (b, i) produces output rows [b·bh, b·bh + bh)
// of image i whole.  It reads once the source rows their vertical taps span ([lo, hi), Pillow's
// ImagingResampleInner order: the horizontal pass covers exactly the rows the vertical one
// reads).  The arithmetic is jpeg_color_resize_h_kernel's + jpeg_resize_v_kernel's, so the
// bytes equal that path's (and PIL decode + Image.resize).
//   0. the planes' 8-row block rows the band reads, copied into LDS with 16-B loads;
//   1. per wave, one source row at a time (no block barrier): the row's colour pixels as RGBX
//      words into the wave's row buffer, then Pillow's horizontal pass from it (one 4-byte LDS
//      read per tap for all three channels) into tmp [rows][TP] (RGB bytes, TP = 3S rounded to 4);
//   2. the vertical pass, which does not care about channels: a lane owns one 4-byte column of
//      tmp, reads one word per tap, keeps 4 sums, and stores the 4 output bytes straight to HBM
//      as one word (a wave writes 256 contiguous bytes of an output row; the band's rows and
//      their taps are wave-uniform).
// dynamic LDS = the largest per-image need (band_layout, host and device alike).
constexpr int BAND_WAVES = 8;  // waves per band block
struct BandLayout {
    int rowbuf, tmp, total, tp;
};
__host__ __device__ inline BandLayout band_layout(int rows, int W, int S, int need_h, int pl) {
    auto al = [](int b) { return (b + 15) & ~15; };
    BandLayout L;
    L.tp = (3 * S + 3) & ~3;
    L.rowbuf = pl;
    L.tmp = pl + (need_h ? al(BAND_WAVES * 2 * ((W + 1) & ~1) * 4) : 0);  // per wave 2 rows × W RGBX words (8-B rows)
    L.total = L.tmp + al(rows * L.tp);
    return L;
}

// LDS bytes of the planes' block rows a band of image rows [y_lo, y_hi) reads (16-B aligned per
// component; offsets written to off[c])
__host__ __device__ inline int band_planes_bytes(const Desc &d, int y_lo, int y_hi, int *off) {
    int total = 0;
    for (int c = 0; c < d.ncomp; ++c) {
        int br0, nbr;
        plane_block_rows(d, c, y_lo, y_hi, &br0, &nbr);
        if (off) off[c] = total;
        total += nbr * d.bw[c] * 64;  // (a multiple of 64)
    }
    return total;
}

constexpr int BAND_NXO = 4;   // output columns per lane held in registers (S <= 256)
constexpr int BAND_MAXV = 8;  // vertical taps held as uniform constants (coefficient tables padded by this)
typedef __attribute__((address_space(3))) void jpeg_lds_void_t;

#if defined(RC_GEMM_ABLATION)
// diagnostic builds: phases of jpeg_band_resize_kernel to skip (1 colour, 2 horizontal, 4 vertical
// math, 8 the plane copy, 16 the vertical pass and its stores; 32 / 64: return after the
// descriptors / after the plane DMA and tap loads), for a per-phase time split
// (tools/jpeg_phase.py); wrong pixels
__device__ int g_band_skip = 0;
#endif

// MAXT > 0 (S <= 64·BAND_NXO): every image's horizontal taps fit MAXT (the coefficient table's
// ksize <= MAXT: 5 for any bicubic upscale, 7 down to a 1.5x downscale): a lane owns output
// columns lane + 64t and keeps their tap offsets and coefficients in registers across the rows
// its wave filters (taps past a column's count have coefficient 0, and their pixel index is
// clamped into the row: exact).  MAXT = 0: the general form (coefficients read per output).
template <int MAXT>
__global__ __launch_bounds__(64 * BAND_WAVES) __attribute__((amdgpu_waves_per_eu(MAXT == 7 ? 7 : 8, 8))) void jpeg_band_resize_kernel(const uint8_t *__restrict__ planes,
                                                              const Desc *__restrict__ descs,
                                                              const RDesc *__restrict__ rdescs, uint8_t *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const Desc d = descs[blockIdx.y];
    const RDesc r = rdescs[blockIdx.y];
    // the coefficient tables through global-address-space pointers: global (not flat) loads,
    // counted by vmcnt alone
    typedef const __attribute__((address_space(1))) int gint_t;
    const gint_t *hb = (const gint_t *)r.hb, *hc = (const gint_t *)r.hc, *vb = (const gint_t *)r.vb,
                 *vc = (const gint_t *)r.vc;
    const int S = r.S, yo0 = (int)blockIdx.x * r.bh;
    if (yo0 >= S) return;  // block-uniform: this image has fewer bands
    const int yo1 = min(S, yo0 + r.bh), nout = yo1 - yo0;
    // wave-uniform in an SGPR: the row-dependent upsampler offsets below then stay scalar
    const int lane = (int)threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    // source rows of the band (relative to r.y0; Pillow's bounds are monotone in the output row)
    const int lo = r.need_v ? vb[2 * yo0] : yo0;
    const int hi = r.need_v ? vb[2 * (yo1 - 1)] + vb[2 * (yo1 - 1) + 1] : yo1;
    const int rows = hi - lo, W = d.W;
#if defined(RC_GEMM_ABLATION)
    if (g_band_skip & 32) return;  // launch + descriptors only
#endif
    // 0. planes (components unrolled with constant indices: a runtime-indexed Desc / offset array
    //    would live in scratch memory, one scratch load per sample read)
    int poff[3], pbr0[3], pnbr[3];
    int pl = 0;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        poff[c] = pl;
        pbr0[c] = pnbr[c] = 0;
        if (c < d.ncomp) {
            plane_block_rows(d, c, r.y0 + lo, r.y0 + hi, &pbr0[c], &pnbr[c]);
            pl += pnbr[c] * d.bw[c] * 64;
        }
    }
    // by LDS-DMA (global_load_lds_dwordx4: no register round trip, every piece of the three
    // planes in flight at once, waited for once below; a wave writes 1 KB of LDS per instruction)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        if (c < d.ncomp) {
            const uint8_t *g = planes + (d.blk0[c] + (int64_t)pbr0[c] * d.bw[c]) * 64;
            const int n16 = pnbr[c] * d.bw[c] * 4;
#if defined(RC_GEMM_ABLATION)
            if (g_band_skip & 8) continue;
#endif
            for (int i0 = wave * 64; i0 < n16; i0 += 64 * BAND_WAVES)
                if (i0 + lane < n16)
                    __builtin_amdgcn_global_load_lds((const void *)(g + 16 * (i0 + lane)),
                                                     (jpeg_lds_void_t *)(lds + poff[c] + 16 * i0), 16, 0, 0);
        }
    }
    const BandLayout L = band_layout(rows, W, S, r.need_h, pl);
    const int TP = L.tp;
    uint32_t *rowbuf = reinterpret_cast<uint32_t *>(lds + L.rowbuf) + wave * 2 * ((W + 1) & ~1);
    uint8_t *tmp = lds + L.tmp;
    // horizontal taps of this lane's output columns (MAXT > 0), kept across its wave's rows and
    // loaded beside the plane DMA (one wait for both): the coefficients and the first tap's pixel
    // xm; tap k reads word xm + k of the row buffer (one address per column, the taps as immediate
    // offsets).  Taps past a column's count have coefficient 0, so the words they read past the
    // row's end (at most MAXT - 1: the next row buffer, or the tmp area after the last) only add 0.
    int cf[MAXT > 0 ? BAND_NXO : 1][MAXT > 0 ? MAXT : 1], xm[MAXT > 0 ? BAND_NXO : 1];
    if constexpr (MAXT > 0) {
        if (r.need_h) {
            __builtin_assume(r.hk >= 1);  // (a resize has taps): no branch around the first load
#pragma unroll
            for (int t = 0; t < BAND_NXO; ++t) {
                const int xo = min(lane + 64 * t, S - 1);
                xm[t] = hb[2 * xo];
                // unguarded loads (the table is padded by BAND_MAXV >= MAXT entries), then the
                // selects: guarded, each load became a branch with its own vmcnt(0)
                int v[MAXT];
#pragma unroll
                for (int k = 0; k < MAXT; ++k) v[k] = hc[xo * r.hk + k];
#pragma unroll
                for (int k = 0; k < MAXT; ++k) cf[t][k] = k < r.hk ? v[k] : 0;
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the plane DMA (and the taps) landed
    __syncthreads();
#if defined(RC_GEMM_ABLATION)
    if (g_band_skip & 64) return;  // + plane DMA and tap loads
#endif
    // jdsample.c's upsampler for one source row y as wave-uniform row offsets into the LDS planes
    // (near / far sample row) and a kind: 0 the sample itself (1x1, or box h2 when the plane is
    // <= 2 samples wide), 1 h1v2, 2 h2v1, 3 h2v2 fancy.  The fancy forms read the neighbour
    // column clamped into the plane, which gives upsampled_t's edge values exactly.
    struct RowTap {
        int bn, bf, kind, rnd, sx, dw1;
    };
    auto row_tap = [&](int c, int y) {
        RowTap t;
        const int rx = d.rx[c], ry = d.ry[c];
        int j = y, far = y;
        t.rnd = 0;
        if (ry == 2) {
            j = y >> 1;
            const int vv = y & 1;
            far = vv == 0 ? max(j - 1, 0) : min(j + 1, d.dh[c] - 1);
            t.rnd = vv == 0 ? 1 : 2;
        }
        auto rowoff = [&](int jj) { return poff[c] + ((jj >> 3) - pbr0[c]) * d.bw[c] * 64 + (jj & 7) * 8; };
        t.bn = rowoff(j);
        t.bf = rowoff(far);
        t.sx = rx == 2 ? 1 : 0;
        t.dw1 = d.dw[c] - 1;
        if (rx == 1) t.kind = ry == 2 ? 1 : 0;
        else if (d.dw[c] <= 2) t.kind = 0;
        else t.kind = ry == 2 ? 3 : 2;
        return t;
    };
    auto col = [](int i) { return ((i >> 3) << 6) + (i & 7); };
    // the component's samples at the pixel pair (2p, 2p + 1): a fancy h2 pair shares its centre
    // column and reads one neighbour each side (3 column reads instead of 4, colsums once)
    // The column offsets of pair p, computed once for every component: c2 = the pair's first
    // full-resolution column, cp / cl / cr = the h2 centre, left and right neighbour (clamped into
    // the plane: component 1's width; component 2's when it differs)
    struct PairCols {
        int c2, cp, cl, cr1, cr2;
    };
    auto pair_cols = [&](int p, const RowTap *tp) {
        PairCols pc;
        pc.c2 = col(2 * p);
        pc.cp = col(p);
        pc.cl = col(max(p - 1, 0));
        const int dwa = tp[d.ncomp > 1 ? 1 : 0].dw1, dwb = tp[d.ncomp > 2 ? 2 : 0].dw1;
        pc.cr1 = col(min(p + 1, dwa));
        pc.cr2 = dwb == dwa ? pc.cr1 : col(min(p + 1, dwb));  // (uniform branch)
        return pc;
    };
    // component sample pair; bn / bf / rnd: this item's row (the wave's two rows differ only there)
    auto sample2 = [&](const RowTap &t, int bn, int bf, int rnd, int p, const PairCols &pc, int cr, int &v0, int &v1) {
        if (t.kind == 0) {
            if (t.sx) {
                v0 = v1 = (int)lds[bn + pc.cp];
            } else {  // x = 2p is even: 2p and 2p + 1 are neighbours within one 8-sample block row
                v0 = (int)lds[bn + pc.c2];
                v1 = (int)lds[bn + pc.c2 + 1];
            }
            return;
        }
        if (t.kind == 1) {
            v0 = (3 * (int)lds[bn + pc.c2] + (int)lds[bf + pc.c2] + rnd) >> 2;
            v1 = (3 * (int)lds[bn + pc.c2 + 1] + (int)lds[bf + pc.c2 + 1] + rnd) >> 2;
            return;
        }
        if (t.kind == 2) {
            const int s0 = 3 * (int)lds[bn + pc.cp];
            v0 = (s0 + (int)lds[bn + pc.cl] + 1) >> 2;
            v1 = (s0 + (int)lds[bn + cr] + 2) >> 2;
            return;
        }
        const int cs0 = 3 * (3 * (int)lds[bn + pc.cp] + (int)lds[bf + pc.cp]);
        const int csl = 3 * (int)lds[bn + pc.cl] + (int)lds[bf + pc.cl];
        const int csr = 3 * (int)lds[bn + cr] + (int)lds[bf + cr];
        v0 = (cs0 + csl + 8) >> 4;
        v1 = (cs0 + csr + 7) >> 4;
    };
    // jdcolor.c ycc_rgb_convert, as ycc_rgb: RGB of one pixel as the word R | G << 8 | B << 16
    auto rgbw = [&](int Y, int cb, int cr) {
        if (d.ncomp == 1) return (uint32_t)__mul24(Y, 0x010101);
        cb -= 128;
        cr -= 128;
        // 24-bit products (|cb|, |cr| <= 128): full-rate v_mad_i32_i24, the same bits
        const int R = min(max(Y + ((__mul24(91881, cr) + 32768) >> 16), 0), 255);
        const int G = min(max(Y + ((__mul24(-22554, cb) + 32768 - __mul24(46802, cr)) >> 16), 0), 255);
        const int B = min(max(Y + ((__mul24(116130, cb) + 32768) >> 16), 0), 255);
        return (uint32_t)R | ((uint32_t)G << 8) | ((uint32_t)B << 16);
    };
    // the pair of row ta (second = false) or tb; only the fields a kind reads are selected
    auto pair_rgb = [&](const RowTap *ta, const RowTap *tb, bool second, int p, uint32_t &w0, uint32_t &w1) {
        const PairCols pc = pair_cols(p, ta);
        auto sel = [&](int c, int &bn, int &bf, int &rnd) __attribute__((always_inline)) {
            bn = second ? tb[c].bn : ta[c].bn;
            bf = ta[c].kind & 1 ? (second ? tb[c].bf : ta[c].bf) : 0;   // kinds 1 and 3 read the far row
            rnd = ta[c].kind == 1 ? (second ? tb[c].rnd : ta[c].rnd) : 0;  // kind 1 rounds by row parity
        };
        int y0, y1, b0 = 0, b1 = 0, r0 = 0, r1 = 0, bn, bf, rnd;
        sel(0, bn, bf, rnd);
        sample2(ta[0], bn, bf, rnd, p, pc, pc.cr1, y0, y1);
        if (d.ncomp != 1) {
            sel(1, bn, bf, rnd);
            sample2(ta[1], bn, bf, rnd, p, pc, pc.cr1, b0, b1);
            sel(2, bn, bf, rnd);
            sample2(ta[2], bn, bf, rnd, p, pc, pc.cr2, r0, r1);
        }
        w0 = rgbw(y0, b0, r0);
        w1 = rgbw(y1, b1, r1);
    };
    // The common 4:2:0 layout (Y full size; Cb, Cr h2v2 fancy-upsampled, as wide as each other and
    // > 2 samples): pair_rgb's arithmetic with the kinds known — the pair's 13 LDS reads (Y as one
    // 16-bit read) issued together, then the sums, instead of a kind dispatch and a wait per
    // component.  Block-uniform; the kinds do not depend on the row.
    auto pair_rgb420 = [&](const RowTap *ta, const RowTap *tb, bool second, int p, uint32_t &w0, uint32_t &w1) {
        const int bny = second ? tb[0].bn : ta[0].bn;
        const int bn1 = second ? tb[1].bn : ta[1].bn, bf1 = second ? tb[1].bf : ta[1].bf;
        const int bn2 = second ? tb[2].bn : ta[2].bn, bf2 = second ? tb[2].bf : ta[2].bf;
        const int c2 = col(2 * p), cp = col(p), cl = col(max(p - 1, 0)), cr = col(min(p + 1, ta[1].dw1));
        const uint32_t yy = *reinterpret_cast<const uint16_t *>(lds + bny + c2);  // 2p, 2p + 1: one block row
        const int n1p = lds[bn1 + cp], f1p = lds[bf1 + cp], n1l = lds[bn1 + cl], f1l = lds[bf1 + cl];
        const int n1r = lds[bn1 + cr], f1r = lds[bf1 + cr];
        const int n2p = lds[bn2 + cp], f2p = lds[bf2 + cp], n2l = lds[bn2 + cl], f2l = lds[bf2 + cl];
        const int n2r = lds[bn2 + cr], f2r = lds[bf2 + cr];
        const int s1 = 3 * (3 * n1p + f1p), s2 = 3 * (3 * n2p + f2p);
        const int b0 = (s1 + 3 * n1l + f1l + 8) >> 4, b1 = (s1 + 3 * n1r + f1r + 7) >> 4;
        const int r0 = (s2 + 3 * n2l + f2l + 8) >> 4, r1 = (s2 + 3 * n2r + f2r + 7) >> 4;
        w0 = rgbw((int)(yy & 255u), b0, r0);
        w1 = rgbw((int)(yy >> 8), b1, r1);
    };
    const bool f420 = d.ncomp == 3 && d.rx[0] == 1 && d.ry[0] == 1 && d.rx[1] == 2 && d.ry[1] == 2 &&
                      d.rx[2] == 2 && d.ry[2] == 2 && d.dw[1] > 2 && d.dw[1] == d.dw[2];
    // 1. colour + horizontal pass, two source rows per wave at a time (no block barrier): the
    //    colour items of both rows are one flat range of pixel pairs (a lone 168-px row is 84 pairs,
    //    2 of 64-lane steps at 66 % use; two rows are 3 steps at 88 %), then the two rows' filter
    //    outputs.  A pair (2p, 2p + 1) of an odd width's last column computes a pixel past the row
    //    (its samples clamped in the plane copy's padding) and does not store it.
#if defined(RC_GEMM_ABLATION)
    const int skip = g_band_skip;
#else
    constexpr int skip = 0;
#endif
    const int npair = (W + 1) >> 1, RW = (W + 1) & ~1;
    for (int r0 = 2 * wave; r0 < rows; r0 += 2 * BAND_WAVES) {
        const int nr = min(2, rows - r0);
        RowTap ta[3], tb[3];
#pragma unroll
        for (int c = 0; c < 3; ++c)
            if (c < d.ncomp) {
                ta[c] = row_tap(c, r.y0 + lo + r0);
                tb[c] = row_tap(c, r.y0 + lo + r0 + nr - 1);
            }
        const int nitems = nr * npair;
        if (!r.need_h) {  // the width already is S: the colour rows are the pass's output
            for (int it = lane; it < nitems; it += 64) {
                const bool second = it >= npair;
                const int p = second ? it - npair : it;
                uint32_t w[2];
                if (f420) pair_rgb420(ta, tb, second, p, w[0], w[1]);
                else pair_rgb(ta, tb, second, p, w[0], w[1]);
                uint8_t *trow = tmp + (r0 + (second ? 1 : 0)) * TP;
                for (int e = 0; e < 2 && 2 * p + e < W; ++e)
                    for (int bb = 0; bb < 3; ++bb) trow[3 * (2 * p + e) + bb] = (uint8_t)(w[e] >> (8 * bb));
            }
            continue;
        }
#pragma unroll 1
        for (int it = lane; it < nitems; it += 64) {
            const bool second = it >= npair;
            const int p = second ? it - npair : it;
            uint32_t w0 = p, w1 = p;
            if (skip & 1) {
            } else if (f420) pair_rgb420(ta, tb, second, p, w0, w1);
            else pair_rgb(ta, tb, second, p, w0, w1);
            uint32_t *rb = rowbuf + (second ? RW : 0) + 2 * p;
            if (2 * p + 1 < W) *reinterpret_cast<uint2 *>(rb) = make_uint2(w0, w1);
            else rb[0] = w0;
        }
        // the row buffers are this wave's alone and LDS executes a wave's accesses in order: no
        // barrier, only no compiler reordering across this point
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        for (int j = 0; j < nr; ++j) {
            const uint32_t *rbuf = rowbuf + j * RW;
            uint8_t *trow = tmp + (r0 + j) * TP;
            if (skip & 2) {
            } else if constexpr (MAXT > 0) {
#pragma unroll
                for (int t = 0; t < BAND_NXO; ++t) {
                    const int xo = lane + 64 * t;
                    if (xo < S) {
                        int a0 = 1 << 21, a1 = 1 << 21, a2 = 1 << 21;
                        const uint32_t *rp = rbuf + xm[t];
#pragma unroll
                        for (int k = 0; k < MAXT; ++k) {
                            const uint32_t w = rp[k];
                            a0 = resample_tap(a0, (int)(w & 255u), cf[t][k]);
                            a1 = resample_tap(a1, (int)((w >> 8) & 255u), cf[t][k]);
                            a2 = resample_tap(a2, (int)(w >> 16), cf[t][k]);
                        }
                        trow[3 * xo] = clip8_22(a0);
                        trow[3 * xo + 1] = clip8_22(a1);
                        trow[3 * xo + 2] = clip8_22(a2);
                    }
                }
            } else {
                for (int xo = lane; xo < S; xo += 64) {
                    const int xmin = hb[2 * xo], xn = hb[2 * xo + 1];
                    const int *c = r.hc + xo * r.hk;
                    int a0 = 1 << 21, a1 = 1 << 21, a2 = 1 << 21;
                    for (int k = 0; k < xn; ++k) {
                        const uint32_t w = rbuf[xmin + k];
                        const int ck = c[k];
                        a0 = resample_tap(a0, (int)(w & 255u), ck);
                        a1 = resample_tap(a1, (int)((w >> 8) & 255u), ck);
                        a2 = resample_tap(a2, (int)(w >> 16), ck);
                    }
                    trow[3 * xo] = clip8_22(a0);
                    trow[3 * xo + 1] = clip8_22(a1);
                    trow[3 * xo + 2] = clip8_22(a2);
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();  // the next rows rewrite the row buffers
    }
    __syncthreads();
    // 2. vertical pass (or, without one, the rows as they are), one output row per wave at a time
    const int rowbytes = 3 * S, nw = TP >> 2;
    const bool words = (rowbytes & 3) == 0;  // out_off = i·S·S·3 is then 4-aligned as well
    uint8_t *gimg = out + r.out_off;
    const uint32_t *t32 = reinterpret_cast<const uint32_t *>(tmp);
    for (int j = wave; j < nout; j += BAND_WAVES) {
        const int yo = yo0 + j;
        uint8_t *grow = gimg + (int64_t)yo * rowbytes;
        if (!r.need_v) {
            for (int cw = lane; cw < nw; cw += 64) {
                const uint32_t v = t32[j * nw + cw];
                if (words) *reinterpret_cast<uint32_t *>(grow + 4 * cw) = v;
                else
                    for (int b = 0; b < 4; ++b)
                        if (4 * cw + b < rowbytes) grow[4 * cw + b] = (uint8_t)(v >> (8 * b));
            }
            continue;
        }
        const int ymin = vb[2 * yo] - lo;
#if defined(RC_GEMM_ABLATION)
        if (g_band_skip & 16) continue;
        const int yn = (g_band_skip & 4) ? 0 : vb[2 * yo + 1];
        const int vk = (g_band_skip & 4) ? 0 : r.vk;
#else
        const int yn = vb[2 * yo + 1];
        const int vk = r.vk;
#endif
        const gint_t *c = vc + yo * r.vk;
        auto store = [&](int cw, int a0, int a1, int a2, int a3) __attribute__((always_inline)) {
            const uint32_t v = (uint32_t)clip8_22(a0) | ((uint32_t)clip8_22(a1) << 8) | ((uint32_t)clip8_22(a2) << 16) |
                               ((uint32_t)clip8_22(a3) << 24);
            if (words) *reinterpret_cast<uint32_t *>(grow + 4 * cw) = v;
            else
                for (int b = 0; b < 4; ++b)
                    if (4 * cw + b < rowbytes) grow[4 * cw + b] = (uint8_t)(v >> (8 * b));
        };
        if (r.vk <= BAND_MAXV) {
            // the row's taps as wave-uniform constants loaded once (the table is padded by
            // BAND_MAXV entries: reads past the row's vk are in bounds), zero past yn, row offsets
            // clamped into the band — not one scalar load per tap per 4-byte column
            int cv[BAND_MAXV], ro[BAND_MAXV];
#pragma unroll
            for (int k = 0; k < BAND_MAXV; ++k) cv[k] = c[k];  // unguarded loads, then the selects
#pragma unroll
            for (int k = 0; k < BAND_MAXV; ++k) {
                cv[k] = k < yn ? cv[k] : 0;
                ro[k] = min(ymin + k, rows - 1) * nw;
            }
            // a column's taps: all T words read first, then the sums (no wait between taps);
            // T = 3, 5, 7 or BAND_MAXV >= vk, the taps past vk reading clamped rows with coefficient 0
            auto vcols = [&](auto tn) __attribute__((always_inline)) {
                constexpr int T = decltype(tn)::value;
                for (int cw = lane; cw < nw; cw += 64) {
                    uint32_t w[T];
#pragma unroll
                    for (int k = 0; k < T; ++k) w[k] = t32[ro[k] + cw];
                    int a0 = 1 << 21, a1 = 1 << 21, a2 = 1 << 21, a3 = 1 << 21;
#pragma unroll
                    for (int k = 0; k < T; ++k) {
                        a0 = resample_tap(a0, (int)(w[k] & 255u), cv[k]);
                        a1 = resample_tap(a1, (int)((w[k] >> 8) & 255u), cv[k]);
                        a2 = resample_tap(a2, (int)((w[k] >> 16) & 255u), cv[k]);
                        a3 = resample_tap(a3, (int)(w[k] >> 24), cv[k]);
                    }
                    store(cw, a0, a1, a2, a3);
                }
            };
            if (vk <= 3) vcols(std::integral_constant<int, 3>{});  // bicubic / bilinear upscale, bilinear to 1.5x
            else if (vk <= 5) vcols(std::integral_constant<int, 5>{});
            else if (vk <= 7) vcols(std::integral_constant<int, 7>{});  // bicubic down to 1.5x
            else vcols(std::integral_constant<int, BAND_MAXV>{});
            continue;
        }
        for (int cw = lane; cw < nw; cw += 64) {
            const uint32_t *q = t32 + ymin * nw + cw;
            int a0 = 1 << 21, a1 = 1 << 21, a2 = 1 << 21, a3 = 1 << 21;
            for (int k = 0; k < yn; ++k) {
                const uint32_t w = q[k * nw];
                const int ck = c[k];
                a0 = resample_tap(a0, (int)(w & 255u), ck);
                a1 = resample_tap(a1, (int)((w >> 8) & 255u), ck);
                a2 = resample_tap(a2, (int)((w >> 16) & 255u), ck);
                a3 = resample_tap(a3, (int)(w >> 24), ck);
            }
            store(cw, a0, a1, a2, a3);
        }
    }
}
}  // namespace jpeg

// Batched decoder: one pinned host staging buffer and its device twin, sized at create.  A call
// lays out [Desc × n | RDesc × n | quant tables × n | qsel × blocks | coefficients × blocks] in
// both (stage_layout) and uploads it with ONE copy (a lone /embed image paid 5 copies, ~5 us each).
struct JpegDecoder {
    int device = 0;
    int max_images = 0;
    int64_t max_blocks = 0;
    uint8_t *h_stage = nullptr, *d_stage = nullptr;
    size_t stage_cap = 0, stage_used = 0;
    // views into the staging (set per call by stage_layout)
    int16_t *h_coef = nullptr;
    int32_t *h_qsel = nullptr;
    uint16_t *h_qtab = nullptr;
    jpeg::Desc *h_desc = nullptr;
    int16_t *d_coef = nullptr;
    int32_t *d_qsel = nullptr;
    uint16_t *d_qtab = nullptr;
    jpeg::Desc *d_desc = nullptr;
    uint8_t *d_planes = nullptr;
    hipEvent_t staged = nullptr;  // the last H2D copy out of the pinned staging
    std::mutex mu;
    // fused decode → resize: per-image plans (in the staging), the two-pass path's horizontal
    // output, Pillow coefficient tables per (size in, size out, filter, y0 shift) built on first use
    jpeg::RDesc *h_rdesc = nullptr, *d_rdesc = nullptr;
    uint8_t *d_tmp = nullptr;
    size_t tmp_bytes = 0;
    struct Coeffs {
        int ksize = 0, first = 0, last = 0;
        int *bounds = nullptr, *coef = nullptr;
        std::vector<int> hbounds;  // host copy of bounds (the band planner reads it)
    };
    std::map<std::tuple<int, int, int, int>, Coeffs> coeffs;
};

}  // namespace rc

struct rc_jpeg_decoder : rc::JpegDecoder {};

using namespace rc;

extern "C" int rc_jpeg_probe(const uint8_t *jpg, int64_t len, rc_jpeg_info *info) {
    return guard([&] {
        RC_REQUIRE(jpg && info, RC_ERR_INVALID, "null argument");
        jpeg::Header hd;
        jpeg::parse(jpg, len, hd);
        jpeg::fill_info(hd, info);
    });
}

extern "C" int rc_jpeg_decode_coefficients(const uint8_t *jpg, int64_t len, int16_t *coef, uint16_t *qtab) {
    return guard([&] {
        RC_REQUIRE(jpg && coef && qtab, RC_ERR_INVALID, "null argument");
        jpeg::Header hd;
        jpeg::parse(jpg, len, hd);
        RC_REQUIRE(hd.supported, RC_ERR_UNSUPPORTED, "JPEG not decodable here: " + hd.why);
        jpeg::decode_coefficients(hd, coef);
        for (int i = 0; i < hd.ncomp; ++i) std::memcpy(qtab + 64 * i, hd.qt[hd.c[i].tq], 64 * sizeof(uint16_t));
    });
}

// The staging layout of a call with n images and nb blocks (256-B aligned regions); with the
// buffers allocated, points the h_* / d_* views at it.  Returns the bytes used.
static size_t stage_layout(JpegDecoder *h, int n, int64_t nb) {
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t o_rdesc = al((size_t)n * sizeof(jpeg::Desc));
    const size_t o_qtab = o_rdesc + al((size_t)n * sizeof(jpeg::RDesc));
    const size_t o_qsel = o_qtab + al((size_t)n * 3 * 128);
    const size_t o_coef = o_qsel + al((size_t)nb * 4);
    const size_t total = o_coef + (size_t)nb * 128;
    if (h->h_stage != nullptr) {
        h->h_desc = reinterpret_cast<jpeg::Desc *>(h->h_stage);
        h->h_rdesc = reinterpret_cast<jpeg::RDesc *>(h->h_stage + o_rdesc);
        h->h_qtab = reinterpret_cast<uint16_t *>(h->h_stage + o_qtab);
        h->h_qsel = reinterpret_cast<int32_t *>(h->h_stage + o_qsel);
        h->h_coef = reinterpret_cast<int16_t *>(h->h_stage + o_coef);
        h->d_desc = reinterpret_cast<jpeg::Desc *>(h->d_stage);
        h->d_rdesc = reinterpret_cast<jpeg::RDesc *>(h->d_stage + o_rdesc);
        h->d_qtab = reinterpret_cast<uint16_t *>(h->d_stage + o_qtab);
        h->d_qsel = reinterpret_cast<int32_t *>(h->d_stage + o_qsel);
        h->d_coef = reinterpret_cast<int16_t *>(h->d_stage + o_coef);
        h->stage_used = total;
    }
    return total;
}

extern "C" int rc_jpeg_decoder_create(int device, int max_images, int64_t max_blocks, rc_jpeg_decoder **out) {
    return guard([&] {
        RC_REQUIRE(out && max_images > 0 && max_blocks > 0, RC_ERR_INVALID, "bad decoder size");
        DeviceScope ds(device);
        auto *h = new rc_jpeg_decoder();
        h->device = device;
        h->max_images = max_images;
        h->max_blocks = max_blocks;
        try {
            h->stage_cap = stage_layout(h, max_images, max_blocks);
            RC_HIP(hipHostMalloc((void **)&h->h_stage, h->stage_cap, hipHostMallocDefault));
            h->d_stage = (uint8_t *)dmalloc(h->stage_cap);
            h->d_planes = (uint8_t *)dmalloc((size_t)max_blocks * 64);
            RC_HIP(hipEventCreateWithFlags(&h->staged, hipEventDisableTiming));
        } catch (...) {
            rc_jpeg_decoder_destroy(h);
            throw;
        }
        *out = h;
    });
}

extern "C" int rc_jpeg_decoder_destroy(rc_jpeg_decoder *h) {
    return guard([&] {
        if (!h) return;
        DeviceScope ds(h->device);
        if (h->staged) (void)hipEventSynchronize(h->staged);
        if (h->h_stage) (void)hipHostFree(h->h_stage);
        dfree(h->d_stage);
        dfree(h->d_planes);
        dfree(h->d_tmp);
        for (auto &kv : h->coeffs) {
            dfree(kv.second.bounds);
            dfree(kv.second.coef);
        }
        if (h->staged) (void)hipEventDestroy(h->staged);
        delete h;
    });
}

// Host Huffman workers per call: RC_JPEG_THREADS if set, else min(16, cores).  In the
// pipelined ingest (embed_jpeg_stream) these threads share the host with the thread
// launching the embed kernels, so fewer than the core count can be faster there.
static int huffman_threads() {
    static const int n = [] {
        if (const char *e = std::getenv("RC_JPEG_THREADS")) {
            const int v = std::atoi(e);
            if (v > 0) return std::min(v, 64);
        }
        return (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    }();
    return n;
}

namespace {

std::atomic<int> g_active_decodes{0};  // decode calls in their Huffman pass right now (any decoder)

// Header parse, host Huffman (threaded) into the pinned staging; fills h->h_desc (rgb_off from
// rgb_offsets, or 0) and the tables.  The caller adds its plans (h_rdesc), then upload_idct.
void stage_host(rc_jpeg_decoder *h, int n, const uint8_t *const *jpgs, const int64_t *lens, const int64_t *rgb_offsets,
                std::vector<jpeg::Header> &hd, int &maxpix, int64_t &nblocks) {
    // headers first (cheap, serial): geometry, block offsets, capacity check
    hd.assign(n, jpeg::Header{});
    std::vector<int64_t> base(n + 1, 0);
    for (int i = 0; i < n; ++i) {
        jpeg::parse(jpgs[i], lens[i], hd[i]);
        RC_REQUIRE(hd[i].supported, RC_ERR_UNSUPPORTED, "JPEG " + std::to_string(i) + " not decodable here: " + hd[i].why);
        base[i + 1] = base[i] + hd[i].blocks;
    }
    RC_REQUIRE(base[n] <= h->max_blocks, RC_ERR_INVALID, "batch exceeds the decoder's max_blocks");
    // the pinned staging is reused: wait for the previous call's upload
    RC_HIP(hipEventSynchronize(h->staged));
    stage_layout(h, n, base[n]);
    // Huffman decode, one image per worker
    std::vector<std::string> errs(n);
    auto work = [&](int i) {
        try {
            jpeg::decode_coefficients(hd[i], h->h_coef + base[i] * 64);
        } catch (const std::exception &e) {
            errs[i] = e.what();
        }
    };
    // concurrent calls (an EmbedderPool decoding per member) split the worker budget
    struct Active {
        int n;
        Active() : n(g_active_decodes.fetch_add(1) + 1) {}
        ~Active() { g_active_decodes.fetch_sub(1); }
    } active;
    const int nthreads = std::max(1, std::min<int>(n, huffman_threads() / active.n));
    if (nthreads == 1) {
        for (int i = 0; i < n; ++i) work(i);
    } else {
        std::vector<std::thread> pool;
        std::atomic<int> next{0};
        for (int t = 0; t < nthreads; ++t)
            pool.emplace_back([&] {
                for (int i; (i = next.fetch_add(1)) < n;) work(i);
            });
        for (auto &t : pool) t.join();
    }
    for (int i = 0; i < n; ++i)
        RC_REQUIRE(errs[i].empty(), RC_ERR_INVALID, "JPEG " + std::to_string(i) + ": " + errs[i]);
    maxpix = 0;
    for (int i = 0; i < n; ++i) {
        const jpeg::Header &H = hd[i];
        jpeg::Desc &d = h->h_desc[i];
        std::memset(&d, 0, sizeof(d));
        d.W = H.width;
        d.H = H.height;
        d.ncomp = H.ncomp;
        for (int c = 0; c < H.ncomp; ++c) {
            d.rx[c] = H.hmax / H.c[c].h;
            d.ry[c] = H.vmax / H.c[c].v;
            d.dw[c] = (int)(((int64_t)H.width * H.c[c].h + H.hmax - 1) / H.hmax);
            d.dh[c] = (int)(((int64_t)H.height * H.c[c].v + H.vmax - 1) / H.vmax);
            d.bw[c] = H.c[c].bw;
            d.blk0[c] = base[i] + H.c[c].blk0;
            std::memcpy(h->h_qtab + (int64_t)(3 * i + c) * 64, H.qt[H.c[c].tq], 128);
            const int64_t nb = (int64_t)H.c[c].bw * H.c[c].bh;
            std::fill(h->h_qsel + d.blk0[c], h->h_qsel + d.blk0[c] + nb, 3 * i + c);
        }
        d.rgb_off = rgb_offsets ? rgb_offsets[i] : 0;
        RC_REQUIRE((int64_t)H.width * H.height < (int64_t)1 << 31, RC_ERR_INVALID, "image too large");
        maxpix = std::max(maxpix, H.width * H.height);
    }
    nblocks = base[n];
}

// One H2D copy of the call's staging (descriptors, plans, tables, coefficients), the event the
// next call waits on before it rewrites the staging, and the IDCT into h->d_planes.
void upload_idct(rc_jpeg_decoder *h, int64_t nb, hipStream_t s) {
    RC_HIP(hipMemcpyAsync(h->d_stage, h->h_stage, h->stage_used, hipMemcpyHostToDevice, s));
    RC_HIP(hipEventRecord(h->staged, s));
    hipLaunchKernelGGL(jpeg::jpeg_idct_kernel, dim3((unsigned)((nb + 7) / 8)), dim3(64), 0, s, h->d_coef, h->d_qsel,
                       h->d_qtab, nb, h->d_planes);
    RC_LAUNCH_CHECK();
}

// Pillow coefficients for in_size -> out_size (bounds shifted down by `shift`), built once.
const rc_jpeg_decoder::Coeffs &resize_coeffs(rc_jpeg_decoder *h, int in_size, int out_size, int resample, int shift) {
    const auto key = std::make_tuple(in_size, out_size, resample, shift);
    auto it = h->coeffs.find(key);
    if (it != h->coeffs.end()) return it->second;
    ResampleCoeffs c = precompute_coeffs(in_size, out_size, resample);
    rc_jpeg_decoder::Coeffs d;
    d.ksize = c.ksize;
    d.first = c.bounds[0];
    d.last = c.bounds[2 * (out_size - 1)] + c.bounds[2 * (out_size - 1) + 1];
    for (int i = 0; i < out_size; ++i) c.bounds[2 * i] -= shift;
    d.hbounds = c.bounds;
    d.bounds = (int *)dmalloc(c.bounds.size() * sizeof(int));
    try {
        // padded by BAND_MAXV zeros: the band kernel reads a row's first BAND_MAXV taps unguarded
        c.coef.resize(c.coef.size() + jpeg::BAND_MAXV, 0);
        d.coef = (int *)dmalloc(c.coef.size() * sizeof(int));
        RC_HIP(hipMemcpy(d.bounds, c.bounds.data(), c.bounds.size() * sizeof(int), hipMemcpyHostToDevice));
        RC_HIP(hipMemcpy(d.coef, c.coef.data(), c.coef.size() * sizeof(int), hipMemcpyHostToDevice));
    } catch (...) {
        dfree(d.bounds);
        dfree(d.coef);
        throw;
    }
    return h->coeffs.emplace(key, d).first->second;
}

}  // namespace

extern "C" int rc_jpeg_decode(rc_jpeg_decoder *h, int n, const uint8_t *const *jpgs, const int64_t *lens,
                              uint8_t *rgb, const int64_t *rgb_offsets, void *stream) {
    return guard([&] {
        RC_REQUIRE(h && jpgs && lens && rgb && rgb_offsets, RC_ERR_INVALID, "null argument");
        RC_REQUIRE(n >= 0 && n <= h->max_images, RC_ERR_INVALID, "batch exceeds the decoder's max_images");
        if (n == 0) return;
        std::lock_guard<std::mutex> lk(h->mu);
        DeviceScope ds(h->device);
        hipStream_t s = (hipStream_t)stream;
        std::vector<jpeg::Header> hd;
        int maxpix = 0;
        int64_t nb = 0;
        stage_host(h, n, jpgs, lens, rgb_offsets, hd, maxpix, nb);
        upload_idct(h, nb, s);
        hipLaunchKernelGGL(jpeg::jpeg_color_kernel, dim3((unsigned)((maxpix + 255) / 256), (unsigned)n), dim3(256), 0, s,
                           h->d_planes, h->d_desc, rgb);
        RC_LAUNCH_CHECK();
    });
}

extern "C" int rc_jpeg_decode_resized(rc_jpeg_decoder *h, int n, const uint8_t *const *jpgs, const int64_t *lens,
                                      int out_size, int resample, uint8_t *out, void *stream) {
    return guard([&] {
        RC_REQUIRE(h && jpgs && lens && out, RC_ERR_INVALID, "null argument");
        RC_REQUIRE(n >= 0 && n <= h->max_images, RC_ERR_INVALID, "batch exceeds the decoder's max_images");
        RC_REQUIRE(out_size >= 1 && out_size <= 4096, RC_ERR_INVALID, "out_size must be in [1, 4096]");
        RC_REQUIRE(resample == RC_RESAMPLE_BICUBIC || resample == RC_RESAMPLE_BILINEAR, RC_ERR_UNSUPPORTED,
                   "resample must be BICUBIC (3) or BILINEAR (2)");
        if (n == 0) return;
        std::lock_guard<std::mutex> lk(h->mu);
        DeviceScope ds(h->device);
        hipStream_t s = (hipStream_t)stream;
        std::vector<jpeg::Header> hd;
        int maxpix = 0;
        int64_t nb = 0;
        stage_host(h, n, jpgs, lens, nullptr, hd, maxpix, nb);
        const int S = out_size;
        int64_t tmp_need = 0;
        int maxrows = 1, maxbands = 1, band_lds = 0, max_hk = 0;
        bool band_ok = true;  // every image's bands fit in LDS: the band kernel, else the two-pass path
        for (int i = 0; i < n; ++i) {
            const int W = hd[i].width, H = hd[i].height;
            jpeg::RDesc &r = h->h_rdesc[i];
            std::memset(&r, 0, sizeof(r));
            r.S = S;
            r.need_h = W != S;
            r.need_v = H != S;
            r.Hs = H;
            if (r.need_h) {
                const auto &ch = resize_coeffs(h, W, S, resample, 0);
                r.hb = ch.bounds;
                r.hc = ch.coef;
                r.hk = ch.ksize;
                max_hk = std::max(max_hk, r.hk);
            }
            const std::vector<int> *vb = nullptr;
            if (r.need_v) {
                const auto &cv = resize_coeffs(h, H, S, resample, 0);
                // ImagingResampleInner: the horizontal pass covers just the rows the vertical one reads
                if (r.need_h) {
                    r.y0 = cv.first;
                    r.Hs = cv.last - cv.first;
                }
                const auto &cvs = r.y0 != 0 ? resize_coeffs(h, H, S, resample, r.y0) : cv;
                r.vb = cvs.bounds;
                r.vc = cvs.coef;
                r.vk = cvs.ksize;
                vb = &cvs.hbounds;
                r.tmp_off = tmp_need;
                tmp_need += (int64_t)r.Hs * S * 3;
            }
            r.out_off = (int64_t)i * S * S * 3;
            maxrows = std::max(maxrows, r.Hs);
            // band height: the tallest band (32 .. 1 output rows) whose LDS (planes' block rows + the
            // 4 waves' colour row buffers + horizontal pass) fits 40 KB (4 blocks per CU), else 64 KB
            // — and no taller than gives the batch >= 128 blocks (a lone /embed image: 224 / 4 = 56
            // bands, not 7-14)
            r.bh = 0;
            int need = 0;
            int bh_max = 32;
            while (bh_max > 4 && (int64_t)n * ((S + bh_max - 1) / bh_max) < 128) bh_max /= 2;
            const jpeg::Desc &dd = h->h_desc[i];
            for (const int cap : {40 * 1024, 64 * 1024}) {
                for (int bh = bh_max; bh >= 1 && r.bh == 0; bh /= 2) {
                    int worst = 0;
                    for (int yo0 = 0; yo0 < S; yo0 += bh) {
                        const int yo1 = std::min(S, yo0 + bh);
                        const int lo = vb ? (*vb)[2 * yo0] : yo0;
                        const int hi = vb ? (*vb)[2 * (yo1 - 1)] + (*vb)[2 * (yo1 - 1) + 1] : yo1;
                        const int pl = jpeg::band_planes_bytes(dd, r.y0 + lo, r.y0 + hi, nullptr);
                        worst = std::max(worst, jpeg::band_layout(hi - lo, W, S, r.need_h, pl).total);
                    }
                    if (worst <= cap) {
                        r.bh = bh;
                        need = worst;
                    }
                }
                if (r.bh) break;
            }
            if (r.bh == 0) band_ok = false;
            else {
                maxbands = std::max(maxbands, (S + r.bh - 1) / r.bh);
                band_lds = std::max(band_lds, need);
            }
        }
        upload_idct(h, nb, s);  // with the plans
        if (band_ok) {
            const dim3 gr((unsigned)maxbands, (unsigned)n);
            // horizontal taps in registers: 5 (any bicubic upscale, e.g. the fixture's 168 -> 224), 7
            // (down to 1.5x), else (or S > 256) the general form
            if (max_hk <= 5 && S <= 64 * jpeg::BAND_NXO)
                hipLaunchKernelGGL(jpeg::jpeg_band_resize_kernel<5>, gr, dim3(64 * jpeg::BAND_WAVES), (size_t)band_lds, s, h->d_planes,
                                   h->d_desc, h->d_rdesc, out);
            else if (max_hk <= 7 && S <= 64 * jpeg::BAND_NXO)
                hipLaunchKernelGGL(jpeg::jpeg_band_resize_kernel<7>, gr, dim3(64 * jpeg::BAND_WAVES), (size_t)band_lds, s, h->d_planes,
                                   h->d_desc, h->d_rdesc, out);
            else
                hipLaunchKernelGGL(jpeg::jpeg_band_resize_kernel<0>, gr, dim3(64 * jpeg::BAND_WAVES), (size_t)band_lds, s, h->d_planes,
                                   h->d_desc, h->d_rdesc, out);
            RC_LAUNCH_CHECK();
            return;
        }
        if ((size_t)tmp_need > h->tmp_bytes) {  // grows geometrically with the largest batch seen
            const size_t want = std::max<size_t>((size_t)tmp_need, 2 * h->tmp_bytes);
            RC_HIP(hipStreamSynchronize(s));
            dfree(h->d_tmp);
            h->d_tmp = nullptr;
            h->tmp_bytes = 0;
            h->d_tmp = (uint8_t *)dmalloc(want);
            h->tmp_bytes = want;
        }
        hipLaunchKernelGGL(jpeg::jpeg_color_resize_h_kernel, dim3((unsigned)maxrows, (unsigned)n), dim3(256), 0, s,
                           h->d_planes, h->d_desc, h->d_rdesc, h->d_tmp, out);
        RC_LAUNCH_CHECK();
        hipLaunchKernelGGL(jpeg::jpeg_resize_v_kernel, dim3((unsigned)((S * S + 255) / 256), (unsigned)n), dim3(256), 0, s,
                           h->d_rdesc, h->d_tmp, out);
        RC_LAUNCH_CHECK();
    });
}

#if defined(RC_GEMM_ABLATION)
// diagnostic builds: the band kernel's phase-skip mask (g_band_skip)
extern "C" int rc_diag_set_band_skip(int mask) {
    return guard([&] { RC_HIP(hipMemcpyToSymbol(HIP_SYMBOL(jpeg::g_band_skip), &mask, sizeof(mask))); });
}
#endif
