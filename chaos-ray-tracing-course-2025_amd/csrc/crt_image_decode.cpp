/*
 * crt_image_decode.cpp — the loader's bitmap decoder, in place of stb_image.
 *
 * The reference loads bitmap textures with `read_stb` (src/core/crt_image_stbi.cpp:16-40):
 * `stbi_load(path, &w, &h, &n, STBI_rgb)`, failure if the file's component
 * count is not 3, then every byte divided by 255.0f.  stb_image is an empty
 * submodule in the reference (vendor/stb, .gitmodules:7-9; pinned commit
 * unknown), so this file restates the published stb_image JPEG algorithm
 * (stable since v2.0x) — the arithmetic that decides the texel bytes:
 *
 *   - Huffman decode of baseline (SOF0/SOF1) and progressive (SOF2) scans with
 *     restart intervals; coefficients are dequantised into int16 with C
 *     truncation ((short)(v * q): baseline at decode time, progressive after
 *     the last scan);
 *   - stb's integer IDCT (`stbi__idct_block`: 12-bit constants f2f(x) =
 *     (int)(x*4096+0.5), column pass >> 10 with +512, row pass >> 17 with
 *     +65536 + (128 << 17), clamp) — its SSE2 form is bit-identical by design;
 *   - chroma upsampling: stb's triangle filter for 2x2 (`resample_row_hv_2`:
 *     3*near+far vertically, (3*a+b+8)>>4 horizontally), (3*a+b+2)>>2 for 2x1
 *     and 1x2, replication otherwise, with stb's near/far row state machine;
 *   - YCbCr -> RGB in 20-bit fixed point with stb's constants
 *     (float2fixed(x) = (int)(x*4096+0.5f) << 8) and its masked Cb term for G
 *     (stb's SIMD converter only runs for 4-byte output, never for STBI_rgb);
 *   - 'R','G','B' component ids, or an Adobe APP14 transform 0 without JFIF,
 *     skip the colour transform.
 *
 * What `read_stb` rejects is rejected here too (component count != 3, i.e.
 * greyscale files), plus what this build does not decode: CMYK/YCCK JPEGs and
 * non-JPEG formats (stb would also read PNG/BMP/TGA/...; no course scene uses
 * them — DESIGN.md §7).  Parity of the decoded bytes with stb itself is
 * unpinned (stb is absent): tests/test_image_decode.py checks the texels
 * against an independent decoder (libjpeg via PIL) within a small tolerance,
 * and the 12-01 renders against the reference's committed PNGs.
 */
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "crt_host.h"

namespace crt_amd {
namespace {

/* natural (row-major) index of the k-th zig-zag coefficient; 15 extra
 * entries so a corrupt run past 63 lands on the last coefficient. */
const uint8_t kDezigzag[64 + 15] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

struct HuffTable {
    bool present = false;
    /* canonical code ranges per length (JPEG Annex F.2.2.3) */
    int32_t mincode[17] = {}, maxcode[18] = {}, valptr[17] = {};
    uint8_t values[256] = {};
};

struct Component {
    int id = 0, h = 1, v = 1, tq = 0;
    int hd = 0, ha = 0;
    int x = 0, y = 0, w2 = 0, h2 = 0;   /* real size, MCU-padded size */
    int dc_pred = 0;
    std::vector<uint8_t> pixels;        /* w2 x h2 IDCT output */
    std::vector<int16_t> coeff;         /* progressive: (w2/8) x (h2/8) blocks of 64 */
    int coeff_w = 0;
};

int clamp_u8(int x) {
    if ((unsigned)x > 255u) return x < 0 ? 0 : 255;
    return x;
}

constexpr int f2f(float x) { return (int)(x * 4096 + 0.5); }

/* One 1-D pass of stb's IDCT over s0..s7 (even/odd parts as jidctint, 12-bit
 * constants); leaves x0..x3 and t0..t3 for the caller's butterfly. */
struct Idct1D {
    int t0, t1, t2, t3, x0, x1, x2, x3;
    Idct1D(int s0, int s1, int s2, int s3, int s4, int s5, int s6, int s7) {
        int p1, p2, p3, p4, p5;
        p2 = s2;
        p3 = s6;
        p1 = (p2 + p3) * f2f(0.5411961f);
        t2 = p1 + p3 * f2f(-1.847759065f);
        t3 = p1 + p2 * f2f(0.765366865f);
        p2 = s0;
        p3 = s4;
        t0 = (p2 + p3) * 4096;
        t1 = (p2 - p3) * 4096;
        x0 = t0 + t3;
        x3 = t0 - t3;
        x1 = t1 + t2;
        x2 = t1 - t2;
        t0 = s7;
        t1 = s5;
        t2 = s3;
        t3 = s1;
        p3 = t0 + t2;
        p4 = t1 + t3;
        p1 = t0 + t3;
        p2 = t1 + t2;
        p5 = (p3 + p4) * f2f(1.175875602f);
        t0 = t0 * f2f(0.298631336f);
        t1 = t1 * f2f(2.053119869f);
        t2 = t2 * f2f(3.072711026f);
        t3 = t3 * f2f(1.501321110f);
        p1 = p5 + p1 * f2f(-0.899976223f);
        p2 = p5 + p2 * f2f(-2.562915447f);
        p3 = p3 * f2f(-1.961570560f);
        p4 = p4 * f2f(-0.390180644f);
        t3 += p1 + p4;
        t2 += p2 + p3;
        t1 += p2 + p4;
        t0 += p1 + p3;
    }
};

void idct_block(uint8_t *out, int stride, const int16_t data[64]) {
    int val[64];
    for (int i = 0; i < 8; ++i) {           /* columns */
        const int16_t *d = data + i;
        int *v = val + i;
        if (d[8] == 0 && d[16] == 0 && d[24] == 0 && d[32] == 0 && d[40] == 0 && d[48] == 0 && d[56] == 0) {
            const int dc = d[0] * 4;
            for (int r = 0; r < 8; ++r) v[8 * r] = dc;
            continue;
        }
        Idct1D k(d[0], d[8], d[16], d[24], d[32], d[40], d[48], d[56]);
        k.x0 += 512; k.x1 += 512; k.x2 += 512; k.x3 += 512;
        v[0] = (k.x0 + k.t3) >> 10;
        v[56] = (k.x0 - k.t3) >> 10;
        v[8] = (k.x1 + k.t2) >> 10;
        v[48] = (k.x1 - k.t2) >> 10;
        v[16] = (k.x2 + k.t1) >> 10;
        v[40] = (k.x2 - k.t1) >> 10;
        v[24] = (k.x3 + k.t0) >> 10;
        v[32] = (k.x3 - k.t0) >> 10;
    }
    for (int i = 0; i < 8; ++i) {           /* rows */
        const int *v = val + 8 * i;
        uint8_t *o = out + (size_t)stride * i;
        Idct1D k(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
        const int bias = 65536 + (128 << 17);
        k.x0 += bias; k.x1 += bias; k.x2 += bias; k.x3 += bias;
        o[0] = (uint8_t)clamp_u8((k.x0 + k.t3) >> 17);
        o[7] = (uint8_t)clamp_u8((k.x0 - k.t3) >> 17);
        o[1] = (uint8_t)clamp_u8((k.x1 + k.t2) >> 17);
        o[6] = (uint8_t)clamp_u8((k.x1 - k.t2) >> 17);
        o[2] = (uint8_t)clamp_u8((k.x2 + k.t1) >> 17);
        o[5] = (uint8_t)clamp_u8((k.x2 - k.t1) >> 17);
        o[3] = (uint8_t)clamp_u8((k.x3 + k.t0) >> 17);
        o[4] = (uint8_t)clamp_u8((k.x3 - k.t0) >> 17);
    }
}

/* upsample one row of a subsampled component (w input samples, hs x vs) */
void resample_row(uint8_t *out, const uint8_t *near, const uint8_t *far, int w, int hs, int vs) {
    if (hs == 1 && vs == 2) {
        for (int i = 0; i < w; ++i) out[i] = (uint8_t)((3 * near[i] + far[i] + 2) >> 2);
        return;
    }
    if (hs == 2 && vs == 1) {
        if (w == 1) { out[0] = out[1] = near[0]; return; }
        out[0] = near[0];
        out[1] = (uint8_t)((near[0] * 3 + near[1] + 2) >> 2);
        int i = 1;
        for (; i < w - 1; ++i) {
            const int n = 3 * near[i] + 2;
            out[i * 2 + 0] = (uint8_t)((n + near[i - 1]) >> 2);
            out[i * 2 + 1] = (uint8_t)((n + near[i + 1]) >> 2);
        }
        /* stb weights the last pair toward in[w-2] (not a triangle filter tap) */
        out[i * 2 + 0] = (uint8_t)((near[w - 2] * 3 + near[w - 1] + 2) >> 2);
        out[i * 2 + 1] = near[w - 1];
        return;
    }
    if (hs == 2 && vs == 2) {
        if (w == 1) { out[0] = out[1] = (uint8_t)((3 * near[0] + far[0] + 2) >> 2); return; }
        int t1 = 3 * near[0] + far[0];
        out[0] = (uint8_t)((t1 + 2) >> 2);
        for (int i = 1; i < w; ++i) {
            const int t0 = t1;
            t1 = 3 * near[i] + far[i];
            out[i * 2 - 1] = (uint8_t)((3 * t0 + t1 + 8) >> 4);
            out[i * 2] = (uint8_t)((3 * t1 + t0 + 8) >> 4);
        }
        out[w * 2 - 1] = (uint8_t)((t1 + 2) >> 2);
        return;
    }
    for (int i = 0; i < w; ++i)
        for (int j = 0; j < hs; ++j) out[i * hs + j] = near[i];
}

inline int float2fixed(float x) { return ((int)(x * 4096.0f + 0.5f)) * 256; }

class Jpeg {
public:
    Jpeg(const uint8_t *p, size_t n) : buf_(p), len_(n) {}
    bool decode(int &w, int &h, int &comps, std::vector<uint8_t> &rgb, std::string &why);

private:
    const uint8_t *buf_;
    size_t len_, pos_ = 0;
    std::string err_;

    uint16_t dequant_[4][64] = {};
    HuffTable dc_[4], ac_[4];
    std::vector<Component> comp_;
    int img_x_ = 0, img_y_ = 0, img_n_ = 0, hmax_ = 1, vmax_ = 1;
    int mcu_x_ = 0, mcu_y_ = 0;
    bool progressive_ = false, jfif_ = false;
    int app14_transform_ = -1, rgb_ids_ = 0;
    int restart_interval_ = 0, todo_ = 0;
    /* current scan */
    int scan_n_ = 0, order_[4] = {0, 0, 0, 0};
    int spec_start_ = 0, spec_end_ = 0, succ_high_ = 0, succ_low_ = 0, eob_run_ = 0;
    /* entropy-coded bit reader: a marker ends the input, zero bits follow */
    uint32_t bits_ = 0;
    int nbits_ = 0;
    int marker_ = -1;
    bool nomore_ = false;

    bool fail(const char *m) {
        if (err_.empty()) err_ = m;
        return false;
    }
    int get8() { return pos_ < len_ ? buf_[pos_++] : 0; }
    int get16() {
        const int a = get8();
        return (a << 8) | get8();
    }
    bool at_eof() const { return pos_ >= len_; }
    void skip(int n) { pos_ = (size_t)n > len_ - pos_ ? len_ : pos_ + (size_t)n; }

    int get_marker() {
        if (marker_ >= 0) {
            const int m = marker_;
            marker_ = -1;
            return m;
        }
        int x = get8();
        if (x != 0xff) return -1;
        while (x == 0xff) x = get8();
        return x;
    }

    void fill() {
        while (nbits_ <= 24) {
            int b = nomore_ ? 0 : get8();
            if (b == 0xff) {
                int c = get8();
                while (c == 0xff) c = get8();
                if (c != 0) {
                    marker_ = c;
                    nomore_ = true;
                    b = 0;
                }
            }
            bits_ |= (uint32_t)b << (24 - nbits_);
            nbits_ += 8;
        }
    }
    int get_bits(int n) {
        if (n == 0) return 0;
        if (nbits_ < n) fill();
        const uint32_t v = bits_ >> (32 - n);
        bits_ <<= n;
        nbits_ -= n;
        return (int)v;
    }
    int get_bit() { return get_bits(1); }
    int extend_receive(int n) {   /* n-bit magnitude category -> signed value */
        const int v = get_bits(n);
        return v < (1 << (n - 1)) ? v - (1 << n) + 1 : v;
    }
    int huff_decode(const HuffTable &t) {
        int code = 0;
        for (int l = 1; l <= 16; ++l) {
            code = (code << 1) | get_bit();
            if (t.maxcode[l] >= 0 && code <= t.maxcode[l]) return t.values[t.valptr[l] + code - t.mincode[l]];
        }
        return -1;
    }
    void reset_scan_state() {
        bits_ = 0;
        nbits_ = 0;
        nomore_ = false;
        marker_ = -1;
        eob_run_ = 0;
        for (Component &c : comp_) c.dc_pred = 0;
        todo_ = restart_interval_ ? restart_interval_ : 0x7fffffff;
    }
    /* after each MCU (or block of a one-component scan): a missing RST marker
     * at the end of an interval ends the scan, keeping what was decoded */
    void restart_step(bool &stop) {
        if (--todo_ > 0) return;
        if (nbits_ < 24) fill();
        if (marker_ < 0xd0 || marker_ > 0xd7) {
            stop = true;
            return;
        }
        reset_scan_state();
    }

    bool process_marker(int m);
    bool frame_header();
    bool scan_header();
    bool decode_block(Component &c, int16_t data[64]);
    bool decode_block_prog_dc(Component &c, int16_t data[64]);
    bool decode_block_prog_ac(Component &c, int16_t data[64]);
    bool entropy_data();
    void finish_progressive();
    void emit_rgb(std::vector<uint8_t> &rgb);
};

bool Jpeg::process_marker(int m) {
    switch (m) {
    case -1:
        return fail("expected marker");
    case 0xdd:   /* DRI */
        if (get16() != 4) return fail("bad DRI length");
        restart_interval_ = get16();
        return true;
    case 0xdb: { /* DQT */
        int L = get16() - 2;
        while (L > 0) {
            const int q = get8(), p = q >> 4, t = q & 15;
            if (p != 0 && p != 1) return fail("bad DQT type");
            if (t > 3) return fail("bad DQT table");
            for (int i = 0; i < 64; ++i) dequant_[t][kDezigzag[i]] = (uint16_t)(p ? get16() : get8());
            L -= p ? 129 : 65;
        }
        return L == 0 ? true : fail("bad DQT length");
    }
    case 0xc4: { /* DHT */
        int L = get16() - 2;
        while (L > 0) {
            const int q = get8(), tc = q >> 4, th = q & 15;
            if (tc > 1 || th > 3) return fail("bad DHT header");
            int counts[17], n = 0;
            for (int i = 1; i <= 16; ++i) {
                counts[i] = get8();
                n += counts[i];
            }
            if (n > 256) return fail("bad DHT header");
            HuffTable &t = tc == 0 ? dc_[th] : ac_[th];
            t.present = true;
            int code = 0, k = 0;
            for (int l = 1; l <= 16; ++l) {
                t.valptr[l] = k;
                t.mincode[l] = code;
                code += counts[l];
                k += counts[l];
                t.maxcode[l] = counts[l] ? code - 1 : -1;
                if (counts[l] && code > (1 << l)) return fail("bad code lengths");
                code <<= 1;
            }
            for (int i = 0; i < n; ++i) t.values[i] = (uint8_t)get8();
            L -= 17 + n;
        }
        return L == 0 ? true : fail("bad DHT length");
    }
    default:
        break;
    }
    if ((m >= 0xe0 && m <= 0xef) || m == 0xfe) {   /* APPn, COM */
        int L = get16();
        if (L < 2) return fail(m == 0xfe ? "bad COM len" : "bad APP len");
        L -= 2;
        if (m == 0xe0 && L >= 5) {
            static const uint8_t tag[5] = {'J', 'F', 'I', 'F', 0};
            bool ok = true;
            for (int i = 0; i < 5; ++i)
                if (get8() != tag[i]) ok = false;
            L -= 5;
            if (ok) jfif_ = true;
        } else if (m == 0xee && L >= 12) {
            static const uint8_t tag[6] = {'A', 'd', 'o', 'b', 'e', 0};
            bool ok = true;
            for (int i = 0; i < 6; ++i)
                if (get8() != tag[i]) ok = false;
            L -= 6;
            if (ok) {
                get8();
                get16();
                get16();
                app14_transform_ = get8();
                L -= 6;
            }
        }
        skip(L);
        return true;
    }
    return fail("unknown marker");
}

bool Jpeg::frame_header() {
    const int Lf = get16();
    if (Lf < 11) return fail("bad SOF len");
    if (get8() != 8) return fail("only 8-bit");
    img_y_ = get16();
    if (img_y_ == 0) return fail("no header height");
    img_x_ = get16();
    if (img_x_ == 0) return fail("0 width");
    img_n_ = get8();
    if (img_n_ != 1 && img_n_ != 3 && img_n_ != 4) return fail("bad component count");
    if (Lf != 8 + 3 * img_n_) return fail("bad SOF len");
    comp_.assign(img_n_, Component());
    static const int rgb_tag[3] = {'R', 'G', 'B'};
    for (int i = 0; i < img_n_; ++i) {
        Component &c = comp_[i];
        c.id = get8();
        if (img_n_ == 3 && c.id == rgb_tag[i]) ++rgb_ids_;
        const int q = get8();
        c.h = q >> 4;
        c.v = q & 15;
        if (c.h < 1 || c.h > 4) return fail("bad H");
        if (c.v < 1 || c.v > 4) return fail("bad V");
        c.tq = get8();
        if (c.tq > 3) return fail("bad TQ");
    }
    for (const Component &c : comp_) {
        hmax_ = c.h > hmax_ ? c.h : hmax_;
        vmax_ = c.v > vmax_ ? c.v : vmax_;
    }
    for (const Component &c : comp_)
        if (hmax_ % c.h != 0 || vmax_ % c.v != 0) return fail("bad subsampling");
    if ((int64_t)img_x_ * img_y_ > ((int64_t)1 << 28)) return fail("too large");
    mcu_x_ = (img_x_ + hmax_ * 8 - 1) / (hmax_ * 8);
    mcu_y_ = (img_y_ + vmax_ * 8 - 1) / (vmax_ * 8);
    for (Component &c : comp_) {
        c.x = (img_x_ * c.h + hmax_ - 1) / hmax_;
        c.y = (img_y_ * c.v + vmax_ - 1) / vmax_;
        c.w2 = mcu_x_ * c.h * 8;
        c.h2 = mcu_y_ * c.v * 8;
        c.pixels.assign((size_t)c.w2 * c.h2, 0);
        if (progressive_) {
            c.coeff_w = c.w2 / 8;
            c.coeff.assign((size_t)c.w2 * c.h2, 0);
        }
    }
    return true;
}

bool Jpeg::scan_header() {
    const int Ls = get16();
    scan_n_ = get8();
    if (scan_n_ < 1 || scan_n_ > 4 || scan_n_ > img_n_) return fail("bad SOS component count");
    if (Ls != 6 + 2 * scan_n_) return fail("bad SOS len");
    for (int i = 0; i < scan_n_; ++i) {
        const int id = get8(), q = get8();
        int which = -1;
        for (int k = 0; k < img_n_; ++k)
            if (comp_[k].id == id) {
                which = k;
                break;
            }
        if (which < 0) return fail("bad SOS component id");
        comp_[which].hd = q >> 4;
        comp_[which].ha = q & 15;
        if (comp_[which].hd > 3 || comp_[which].ha > 3) return fail("bad huffman table");
        order_[i] = which;
    }
    spec_start_ = get8();
    spec_end_ = get8();
    const int aa = get8();
    succ_high_ = aa >> 4;
    succ_low_ = aa & 15;
    if (progressive_) {
        if (spec_start_ > 63 || spec_end_ > 63 || spec_start_ > spec_end_ || succ_high_ > 13 || succ_low_ > 13)
            return fail("bad SOS");
    } else {
        if (spec_start_ != 0 || succ_high_ != 0 || succ_low_ != 0) return fail("bad SOS");
        spec_end_ = 63;
    }
    return true;
}

bool Jpeg::decode_block(Component &c, int16_t data[64]) {
    const HuffTable &hd = dc_[c.hd], &ha = ac_[c.ha];
    if (!hd.present || !ha.present) return fail("missing huffman table");
    const uint16_t *dq = dequant_[c.tq];
    const int t = huff_decode(hd);
    if (t < 0 || t > 15) return fail("bad huffman code");
    std::memset(data, 0, 64 * sizeof(int16_t));
    const int diff = t ? extend_receive(t) : 0;
    const int dc = c.dc_pred + diff;
    c.dc_pred = dc;
    data[0] = (int16_t)(dc * dq[0]);
    int k = 1;
    do {
        const int rs = huff_decode(ha);
        if (rs < 0) return fail("bad huffman code");
        const int s = rs & 15, r = rs >> 4;
        if (s == 0) {
            if (rs != 0xf0) break;   /* end of block */
            k += 16;
        } else {
            k += r;
            const int zig = kDezigzag[k++];
            data[zig] = (int16_t)(extend_receive(s) * dq[zig]);
        }
    } while (k < 64);
    return true;
}

bool Jpeg::decode_block_prog_dc(Component &c, int16_t data[64]) {
    if (spec_end_ != 0) return fail("can't merge dc and ac");
    if (succ_high_ == 0) {
        if (!dc_[c.hd].present) return fail("missing huffman table");
        std::memset(data, 0, 64 * sizeof(int16_t));
        const int t = huff_decode(dc_[c.hd]);
        if (t < 0 || t > 15) return fail("bad huffman code");
        const int diff = t ? extend_receive(t) : 0;
        const int dc = c.dc_pred + diff;
        c.dc_pred = dc;
        data[0] = (int16_t)(dc * (1 << succ_low_));
    } else if (get_bit()) {
        data[0] = (int16_t)(data[0] + (1 << succ_low_));
    }
    return true;
}

bool Jpeg::decode_block_prog_ac(Component &c, int16_t data[64]) {
    if (spec_start_ == 0) return fail("can't merge dc and ac");
    const HuffTable &ha = ac_[c.ha];
    if (!ha.present) return fail("missing huffman table");
    if (succ_high_ == 0) {
        const int shift = succ_low_;
        if (eob_run_) {
            --eob_run_;
            return true;
        }
        int k = spec_start_;
        do {
            const int rs = huff_decode(ha);
            if (rs < 0) return fail("bad huffman code");
            const int s = rs & 15, r = rs >> 4;
            if (s == 0) {
                if (r < 15) {
                    eob_run_ = 1 << r;
                    if (r) eob_run_ += get_bits(r);
                    --eob_run_;
                    break;
                }
                k += 16;
            } else {
                k += r;
                const int zig = kDezigzag[k++];
                data[zig] = (int16_t)(extend_receive(s) * (1 << shift));
            }
        } while (k <= spec_end_);
        return true;
    }
    /* refinement scan */
    const int16_t bit = (int16_t)(1 << succ_low_);
    auto refine = [&](int16_t *p) {
        if (get_bit() && (*p & bit) == 0) *p = (int16_t)(*p > 0 ? *p + bit : *p - bit);
    };
    if (eob_run_) {
        --eob_run_;
        for (int k = spec_start_; k <= spec_end_; ++k) {
            int16_t *p = &data[kDezigzag[k]];
            if (*p != 0) refine(p);
        }
        return true;
    }
    int k = spec_start_;
    do {
        const int rs = huff_decode(ha);
        if (rs < 0) return fail("bad huffman code");
        int s = rs & 15, r = rs >> 4;
        if (s == 0) {
            if (r < 15) {
                eob_run_ = (1 << r) - 1;
                if (r) eob_run_ += get_bits(r);
                r = 64;   /* force end of block */
            }
            /* r == 15: a run of 15 zeros, then a zero coefficient */
        } else {
            if (s != 1) return fail("bad huffman code");
            s = get_bit() ? bit : -bit;
        }
        while (k <= spec_end_) {
            int16_t *p = &data[kDezigzag[k++]];
            if (*p != 0) {
                refine(p);
            } else {
                if (r == 0) {
                    *p = (int16_t)s;
                    break;
                }
                --r;
            }
        }
    } while (k <= spec_end_);
    return true;
}

bool Jpeg::entropy_data() {
    reset_scan_state();
    bool stop = false;
    int16_t block[64];
    if (scan_n_ == 1) {   /* non-interleaved: the component's own block grid */
        Component &c = comp_[order_[0]];
        const int w = (c.x + 7) >> 3, h = (c.y + 7) >> 3;
        for (int j = 0; j < h && !stop; ++j)
            for (int i = 0; i < w && !stop; ++i) {
                if (!progressive_) {
                    if (!decode_block(c, block)) return false;
                    idct_block(c.pixels.data() + (size_t)c.w2 * j * 8 + i * 8, c.w2, block);
                } else {
                    int16_t *data = c.coeff.data() + 64 * ((size_t)i + (size_t)j * c.coeff_w);
                    if (!(spec_start_ == 0 ? decode_block_prog_dc(c, data) : decode_block_prog_ac(c, data)))
                        return false;
                }
                restart_step(stop);
            }
        return true;
    }
    for (int j = 0; j < mcu_y_ && !stop; ++j)
        for (int i = 0; i < mcu_x_ && !stop; ++i) {
            for (int k = 0; k < scan_n_; ++k) {
                Component &c = comp_[order_[k]];
                for (int y = 0; y < c.v; ++y)
                    for (int x = 0; x < c.h; ++x) {
                        const int x2 = i * c.h + x, y2 = j * c.v + y;
                        if (!progressive_) {
                            if (!decode_block(c, block)) return false;
                            idct_block(c.pixels.data() + (size_t)c.w2 * y2 * 8 + x2 * 8, c.w2, block);
                        } else {
                            int16_t *data = c.coeff.data() + 64 * ((size_t)x2 + (size_t)y2 * c.coeff_w);
                            if (!decode_block_prog_dc(c, data)) return false;
                        }
                    }
            }
            restart_step(stop);
        }
    return true;
}

void Jpeg::finish_progressive() {
    for (Component &c : comp_) {
        const int w = (c.x + 7) >> 3, h = (c.y + 7) >> 3;
        const uint16_t *dq = dequant_[c.tq];
        for (int j = 0; j < h; ++j)
            for (int i = 0; i < w; ++i) {
                int16_t *data = c.coeff.data() + 64 * ((size_t)i + (size_t)j * c.coeff_w);
                for (int k = 0; k < 64; ++k) data[k] = (int16_t)(data[k] * dq[k]);
                idct_block(c.pixels.data() + (size_t)c.w2 * j * 8 + i * 8, c.w2, data);
            }
    }
}

void Jpeg::emit_rgb(std::vector<uint8_t> &rgb) {
    rgb.assign((size_t)img_x_ * img_y_ * 3, 0);
    struct Res {
        int hs, vs, ystep, ypos, w_lores;
        const uint8_t *line0, *line1;
        std::vector<uint8_t> buf;
    };
    Res res[3];
    for (int k = 0; k < 3; ++k) {
        Res &r = res[k];
        const Component &c = comp_[k];
        r.hs = hmax_ / c.h;
        r.vs = vmax_ / c.v;
        r.ystep = r.vs >> 1;
        r.w_lores = (img_x_ + r.hs - 1) / r.hs;
        r.ypos = 0;
        r.line0 = r.line1 = c.pixels.data();
        r.buf.assign((size_t)r.w_lores * r.hs + 3, 0);
    }
    const bool is_rgb = rgb_ids_ == 3 || (app14_transform_ == 0 && !jfif_);
    const int cr_r = float2fixed(1.40200f), cr_g = -float2fixed(0.71414f);
    const int cb_g = -float2fixed(0.34414f), cb_b = float2fixed(1.77200f);
    const uint8_t *row[3];
    for (int j = 0; j < img_y_; ++j) {
        for (int k = 0; k < 3; ++k) {
            Res &r = res[k];
            const bool y_bot = r.ystep >= (r.vs >> 1);
            const uint8_t *near = y_bot ? r.line1 : r.line0, *far = y_bot ? r.line0 : r.line1;
            if (r.hs == 1 && r.vs == 1) {
                row[k] = near;
            } else {
                resample_row(r.buf.data(), near, far, r.w_lores, r.hs, r.vs);
                row[k] = r.buf.data();
            }
            if (++r.ystep >= r.vs) {
                r.ystep = 0;
                r.line0 = r.line1;
                if (++r.ypos < comp_[k].y) r.line1 += comp_[k].w2;
            }
        }
        uint8_t *out = rgb.data() + (size_t)3 * img_x_ * j;
        for (int i = 0; i < img_x_; ++i, out += 3) {
            if (is_rgb) {
                out[0] = row[0][i];
                out[1] = row[1][i];
                out[2] = row[2][i];
                continue;
            }
            const int y_fixed = (row[0][i] << 20) + (1 << 19);
            const int cr = row[2][i] - 128, cb = row[1][i] - 128;
            const int r = y_fixed + cr * cr_r;
            const int g = y_fixed + cr * cr_g + (int)((unsigned)(cb * cb_g) & 0xffff0000u);
            const int b = y_fixed + cb * cb_b;
            out[0] = (uint8_t)clamp_u8(r >> 20);
            out[1] = (uint8_t)clamp_u8(g >> 20);
            out[2] = (uint8_t)clamp_u8(b >> 20);
        }
    }
}

bool Jpeg::decode(int &w, int &h, int &comps, std::vector<uint8_t> &rgb, std::string &why) {
    auto failed = [&]() {
        why = err_.empty() ? "corrupt JPEG" : err_;
        return false;
    };
    if (get_marker() != 0xd8) {
        fail("no SOI");
        return failed();
    }
    int m = get_marker();
    while (m != 0xc0 && m != 0xc1 && m != 0xc2) {
        if (!process_marker(m)) return failed();
        m = get_marker();
        while (m == -1) {
            if (at_eof()) {
                fail("no SOF");
                return failed();
            }
            m = get_marker();
        }
    }
    progressive_ = m == 0xc2;
    if (!frame_header()) return failed();
    comps = img_n_ >= 3 ? 3 : 1;   /* what stbi_load reports as the file's component count */
    if (img_n_ != 3) {
        fail(img_n_ == 1 ? "greyscale image (read_stb needs 3 components)" : "CMYK/YCCK JPEG not supported");
        return failed();
    }
    bool truncated = false;
    m = get_marker();
    while (m != 0xd9) {   /* EOI */
        if (m == 0xda) {  /* SOS */
            if (!scan_header() || !entropy_data()) return failed();
            if (marker_ < 0) {   /* skip trailing bytes up to the next marker */
                while (pos_ < len_) {
                    if (buf_[pos_] == 0xff && pos_ + 1 < len_ && buf_[pos_ + 1] != 0 && buf_[pos_ + 1] != 0xff) break;
                    ++pos_;
                }
            }
            m = get_marker();
            if (m >= 0xd0 && m <= 0xd7) m = get_marker();
        } else if (m == 0xdc) {   /* DNL */
            const int Ld = get16(), NL = get16();
            if (Ld != 4 || NL != img_y_) {
                fail("bad DNL");
                return failed();
            }
            m = get_marker();
        } else {
            if (!process_marker(m)) {   /* stb keeps what was decoded so far */
                truncated = true;
                break;
            }
            m = get_marker();
        }
    }
    if (progressive_ && !truncated) finish_progressive();
    emit_rgb(rgb);
    w = img_x_;
    h = img_y_;
    return true;
}

}  // namespace

bool decode_image_rgb8(const uint8_t *bytes, size_t len, int &w, int &h, int &comps, std::vector<uint8_t> &rgb,
                       std::string &why) {
    w = h = comps = 0;
    if (!bytes || len < 4 || bytes[0] != 0xff || bytes[1] != 0xd8) {
        why = "not a JPEG file (this build decodes JPEG bitmaps only)";
        return false;
    }
    Jpeg j(bytes, len);
    return j.decode(w, h, comps, rgb, why);
}

}  // namespace crt_amd

extern "C" int crt_image_decode_rgb8(const uint8_t *bytes, size_t len, int32_t *width, int32_t *height,
                                     int32_t *file_components, uint8_t *rgb_out, size_t cap) {
    using namespace crt_amd;
    if (!bytes || !width || !height) return set_error(CRT_E_INVALID, "null argument");
    int w = 0, h = 0, comps = 0;
    std::vector<uint8_t> rgb;
    std::string why;
    const bool ok = decode_image_rgb8(bytes, len, w, h, comps, rgb, why);
    if (file_components) *file_components = comps;
    if (!ok) return set_error(CRT_E_UNSUPPORTED, "image decode: " + why);
    *width = w;
    *height = h;
    if (rgb_out) {
        if (cap < rgb.size()) return set_error(CRT_E_INVALID, "rgb_out too small");
        std::memcpy(rgb_out, rgb.data(), rgb.size());
    }
    return CRT_OK;
}
