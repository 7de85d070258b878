// imagedec.cpp — JPEG and PNG decoding for image textures (imagedec.h).  Own implementation of the two standards;
// the numeric conventions where the standards leave a choice are stb_image v2.27's (the reference's decoder):
//   * JPEG coefficients are kept as int16 (products with the quantizer wrap as a C short does), the inverse DCT is the
//     integer "islow" transform with stb's constants, 2 extra bits after the column pass and the +128 level shift in the
//     row pass's rounding bias, the color transform is stb's 20-bit fixed point (Cb's G term truncated to 16 fractional
//     bits), and chroma is upsampled with stb's triangle filters;
//   * PNG 16-bit samples keep their high byte; 1/2/4-bit gray samples are scaled by 0xff/0x55/0x11.
#include "imagedec.h"

#include <zlib.h>

#include <algorithm>
#include <cstring>
#include <fstream>
#include <iterator>
#include <stdexcept>

namespace art {
namespace {

// ================================================================================================ JPEG
[[noreturn]] void jbad(const std::string& what) { throw std::runtime_error("JPEG: " + what); }

// natural (row-major) index of the k-th coefficient in zigzag order (T.81 Figure A.6)
constexpr uint8_t kNatural[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
                                  41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                                  30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct Huffman {  // canonical code (T.81 Annex C / F.2.2.3)
    bool defined = false;
    int32_t mincode[17] = {}, maxcode[17] = {}, valptr[17] = {};
    uint8_t vals[256] = {};
    void build(const uint8_t counts[16], const uint8_t* v, int n) {
        std::memcpy(vals, v, static_cast<size_t>(n));
        int32_t code = 0, k = 0;
        for (int len = 1; len <= 16; ++len) {
            valptr[len] = k;
            mincode[len] = code;
            code += counts[len - 1];
            k += counts[len - 1];
            maxcode[len] = counts[len - 1] ? code - 1 : -1;
            if (code > (1 << len)) jbad("bad huffman table");
            code <<= 1;
        }
        defined = true;
    }
};

// Entropy-coded segment reader: bytes, 0xFF00 stuffing; a marker ends the data (zeros are fed after it).
struct BitReader {
    const uint8_t* p;
    const uint8_t* end;
    uint32_t buf = 0;
    int nbits = 0;
    int marker = -1;  // a marker met inside the entropy data, not yet consumed
    int byte() {
        if (marker >= 0 || p >= end) return 0;
        const int b = *p++;
        if (b != 0xFF) return b;
        int m = p < end ? *p : 0;
        while (m == 0xFF && p + 1 < end) m = *++p;  // fill bytes
        if (m == 0x00) {
            ++p;
            return 0xFF;
        }
        ++p;
        marker = m;
        return 0;
    }
    int bit() {
        if (nbits == 0) {
            buf = static_cast<uint32_t>(byte());
            nbits = 8;
        }
        --nbits;
        return static_cast<int>((buf >> nbits) & 1u);
    }
    int bits(int n) {
        int v = 0;
        for (int i = 0; i < n; ++i) v = (v << 1) | bit();
        return v;
    }
    int decode(const Huffman& h) {
        if (!h.defined) jbad("undefined huffman table");
        int32_t code = 0;
        for (int len = 1; len <= 16; ++len) {
            code = (code << 1) | bit();
            if (code <= h.maxcode[len]) return h.vals[h.valptr[len] + code - h.mincode[len]];
        }
        jbad("bad huffman code");
    }
    int extend(int s) {  // RECEIVE(s) + EXTEND (F.2.2.1)
        if (s == 0) return 0;
        const int v = bits(s);
        return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v;
    }
    // restart marker between intervals: drop the partial byte, expect RSTn
    void restart() {
        nbits = 0;
        buf = 0;
        if (marker < 0) {
            while (p < end && *p != 0xFF) ++p;  // tolerate junk before the marker
            while (p < end && *p == 0xFF) ++p;
            if (p < end) marker = *p++;
        }
        if (marker < 0xD0 || marker > 0xD7) jbad("missing restart marker");
        marker = -1;
    }
};

struct Component {
    int id = 0, h = 1, v = 1, tq = 0;
    int td = 0, ta = 0;
    int x = 0, y = 0;    // effective samples
    int w2 = 0, h2 = 0;  // MCU-padded plane size
    int dc_pred = 0;
    std::vector<int16_t> coeff;  // (w2/8) x (h2/8) blocks of 64, natural order
    std::vector<uint8_t> plane;  // w2 x h2 samples after the IDCT
};

inline uint8_t clamp8(int x) { return static_cast<uint8_t>(x < 0 ? 0 : (x > 255 ? 255 : x)); }

// Integer inverse DCT (the IJG "islow" 1-D transform, constants scaled by 2^12) as stb_image's stbi__idct_block does
// it: columns first with two extra fraction bits ((x + 512) >> 10), then rows with the combined scale, the rounding
// and the +128 level shift in one bias ((x + 65536 + (128 << 17)) >> 17), clamped to 0..255.
inline int f2f(double x) { return static_cast<int>(x * 4096 + 0.5); }
struct Idct1d {
    int t0, t1, t2, t3, x0, x1, x2, x3;
    Idct1d(int s0, int s1, int s2, int s3, int s4, int s5, int s6, int s7) {
        static const int c0 = f2f(0.5411961f), c1 = f2f(-1.847759065f), c2 = f2f(0.765366865f), c3 = f2f(1.175875602f),
                         c4 = f2f(0.298631336f), c5 = f2f(2.053119869f), c6 = f2f(3.072711026f), c7 = f2f(1.501321110f),
                         c8 = f2f(-0.899976223f), c9 = f2f(-2.562915447f), c10 = f2f(-1.961570560f), c11 = f2f(-0.390180644f);
        // even part
        int p2 = s2, p3 = s6;
        int p1 = (p2 + p3) * c0;
        t2 = p1 + p3 * c1;
        t3 = p1 + p2 * c2;
        p2 = s0;
        p3 = s4;
        t0 = (p2 + p3) * 4096;
        t1 = (p2 - p3) * 4096;
        x0 = t0 + t3;
        x3 = t0 - t3;
        x1 = t1 + t2;
        x2 = t1 - t2;
        // odd part
        t0 = s7;
        t1 = s5;
        t2 = s3;
        t3 = s1;
        p3 = t0 + t2;
        int p4 = t1 + t3;
        p1 = t0 + t3;
        p2 = t1 + t2;
        const int p5 = (p3 + p4) * c3;
        t0 = t0 * c4;
        t1 = t1 * c5;
        t2 = t2 * c6;
        t3 = t3 * c7;
        p1 = p5 + p1 * c8;
        p2 = p5 + p2 * c9;
        p3 = p3 * c10;
        p4 = p4 * c11;
        t3 += p1 + p4;
        t2 += p2 + p3;
        t1 += p2 + p4;
        t0 += p1 + p3;
    }
};
void idct_block(const int16_t* d, uint8_t* out, int stride) {
    int v[64];
    for (int i = 0; i < 8; ++i) {
        const int16_t* c = d + i;
        if (c[8] == 0 && c[16] == 0 && c[24] == 0 && c[32] == 0 && c[40] == 0 && c[48] == 0 && c[56] == 0) {
            const int dc = c[0] * 4;  // the same value as the full transform of a DC-only column
            for (int r = 0; r < 8; ++r) v[i + 8 * r] = dc;
            continue;
        }
        Idct1d t(c[0], c[8], c[16], c[24], c[32], c[40], c[48], c[56]);
        t.x0 += 512;
        t.x1 += 512;
        t.x2 += 512;
        t.x3 += 512;
        v[i + 0] = (t.x0 + t.t3) >> 10;
        v[i + 56] = (t.x0 - t.t3) >> 10;
        v[i + 8] = (t.x1 + t.t2) >> 10;
        v[i + 48] = (t.x1 - t.t2) >> 10;
        v[i + 16] = (t.x2 + t.t1) >> 10;
        v[i + 40] = (t.x2 - t.t1) >> 10;
        v[i + 24] = (t.x3 + t.t0) >> 10;
        v[i + 32] = (t.x3 - t.t0) >> 10;
    }
    for (int r = 0; r < 8; ++r) {
        const int* s = v + 8 * r;
        Idct1d t(s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7]);
        const int bias = 65536 + (128 << 17);
        t.x0 += bias;
        t.x1 += bias;
        t.x2 += bias;
        t.x3 += bias;
        uint8_t* o = out + static_cast<size_t>(r) * stride;
        o[0] = clamp8((t.x0 + t.t3) >> 17);
        o[7] = clamp8((t.x0 - t.t3) >> 17);
        o[1] = clamp8((t.x1 + t.t2) >> 17);
        o[6] = clamp8((t.x1 - t.t2) >> 17);
        o[2] = clamp8((t.x2 + t.t1) >> 17);
        o[5] = clamp8((t.x2 - t.t1) >> 17);
        o[3] = clamp8((t.x3 + t.t0) >> 17);
        o[4] = clamp8((t.x3 - t.t0) >> 17);
    }
}

struct Jpeg {
    Jpeg(const uint8_t* b, const uint8_t* e) : p(b), end(e) {}
    const uint8_t* p;
    const uint8_t* end;
    int W = 0, H = 0, ncomp = 0;
    bool progressive = false, jfif = false;
    int adobe_transform = -1;
    int restart_interval = 0;
    int hmax = 1, vmax = 1, mcux = 0, mcuy = 0;
    Component comp[4];
    uint16_t quant[4][64] = {};
    Huffman dc[4], ac[4];
    // scan state
    int scan_n = 0, order[4] = {}, ss = 0, se = 63, ah = 0, al = 0;
    int eob_run = 0;

    int u8() {
        if (p >= end) jbad("truncated file");
        return *p++;
    }
    int u16() {
        const int a = u8();
        return (a << 8) | u8();
    }
    int next_marker() {  // the next marker at p (skipping fill bytes and anything that is not a marker)
        while (p < end) {
            if (*p++ != 0xFF) continue;
            while (p < end && *p == 0xFF) ++p;
            if (p >= end) break;
            const int m = *p++;
            if (m != 0) return m;
        }
        return -1;
    }

    void frame(int m) {
        progressive = m == 0xC2;
        const int len = u16();
        if (u8() != 8) jbad("only 8-bit samples are supported");
        H = u16();
        W = u16();
        ncomp = u8();
        if (W == 0 || H == 0) jbad("zero image size (DNL-defined height is not supported)");
        if (ncomp != 1 && ncomp != 3 && ncomp != 4) jbad("bad component count");
        if (len != 8 + 3 * ncomp) jbad("bad SOF length");
        for (int i = 0; i < ncomp; ++i) {
            Component& c = comp[i];
            c.id = u8();
            const int hv = u8();
            c.h = hv >> 4;
            c.v = hv & 15;
            c.tq = u8();
            if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4 || c.tq > 3) jbad("bad component parameters");
            hmax = std::max(hmax, c.h);
            vmax = std::max(vmax, c.v);
        }
        for (int i = 0; i < ncomp; ++i)
            if (hmax % comp[i].h || vmax % comp[i].v) jbad("non-integer sampling ratio");
        mcux = (W + 8 * hmax - 1) / (8 * hmax);
        mcuy = (H + 8 * vmax - 1) / (8 * vmax);
        for (int i = 0; i < ncomp; ++i) {
            Component& c = comp[i];
            c.x = (W * c.h + hmax - 1) / hmax;
            c.y = (H * c.v + vmax - 1) / vmax;
            c.w2 = mcux * c.h * 8;
            c.h2 = mcuy * c.v * 8;
            c.coeff.assign(static_cast<size_t>(c.w2) * c.h2, 0);
            c.plane.assign(static_cast<size_t>(c.w2) * c.h2, 0);
        }
    }
    void dqt() {
        int len = u16() - 2;
        while (len > 0) {
            const int q = u8(), prec = q >> 4, t = q & 15;
            if (prec > 1 || t > 3) jbad("bad DQT");
            for (int i = 0; i < 64; ++i) quant[t][kNatural[i]] = static_cast<uint16_t>(prec ? u16() : u8());
            len -= prec ? 129 : 65;
        }
        if (len != 0) jbad("bad DQT length");
    }
    void dht() {
        int len = u16() - 2;
        while (len > 0) {
            const int q = u8(), cls = q >> 4, id = q & 15;
            if (cls > 1 || id > 3) jbad("bad DHT");
            uint8_t counts[16];
            int n = 0;
            for (int i = 0; i < 16; ++i) n += counts[i] = static_cast<uint8_t>(u8());
            if (n > 256 || end - p < n) jbad("bad DHT");
            (cls ? ac[id] : dc[id]).build(counts, p, n);
            p += n;
            len -= 17 + n;
        }
        if (len != 0) jbad("bad DHT length");
    }
    void app(int m) {
        int len = u16() - 2;
        if (len < 0 || end - p < len) jbad("bad APP/COM length");
        if (m == 0xE0 && len >= 5 && std::memcmp(p, "JFIF\0", 5) == 0) jfif = true;
        if (m == 0xEE && len >= 12 && std::memcmp(p, "Adobe\0", 6) == 0) adobe_transform = p[11];
        p += len;
    }

    void scan_header() {
        const int len = u16();
        scan_n = u8();
        if (scan_n < 1 || scan_n > ncomp || len != 6 + 2 * scan_n) jbad("bad SOS");
        for (int i = 0; i < scan_n; ++i) {
            const int id = u8(), t = u8();
            int which = 0;
            while (which < ncomp && comp[which].id != id) ++which;
            if (which == ncomp) jbad("SOS names an unknown component");
            comp[which].td = t >> 4;
            comp[which].ta = t & 15;
            if (comp[which].td > 3 || comp[which].ta > 3) jbad("bad SOS table");
            order[i] = which;
        }
        ss = u8();
        se = u8();
        const int a = u8();
        ah = a >> 4;
        al = a & 15;
        if (progressive) {
            if (ss > 63 || se > 63 || ss > se || ah > 13 || al > 13) jbad("bad progressive SOS");
            if ((ss == 0) != (se == 0)) jbad("a progressive scan mixes DC and AC");
            if (ss > 0 && scan_n != 1) jbad("interleaved progressive AC scan");
        } else {
            if (ss != 0 || ah != 0 || al != 0) jbad("bad sequential SOS");
            se = 63;
        }
    }

    int16_t* block(Component& c, int bx, int by) { return c.coeff.data() + 64 * (static_cast<size_t>(by) * (c.w2 / 8) + bx); }

    void block_sequential(BitReader& br, Component& c, int16_t* d) {
        const int t = br.decode(dc[c.td]);
        if (t > 15) jbad("bad DC magnitude");
        c.dc_pred += br.extend(t);
        const uint16_t* q = quant[c.tq];
        d[0] = static_cast<int16_t>(c.dc_pred * q[0]);  // stb: (short)(dc * dequant[0])
        for (int k = 1; k < 64;) {
            const int rs = br.decode(ac[c.ta]), r = rs >> 4, s = rs & 15;
            if (s == 0) {
                if (rs != 0xF0) break;  // EOB
                k += 16;
                continue;
            }
            k += r;
            if (k > 63) jbad("AC coefficient past the block");
            const int z = kNatural[k++];
            d[z] = static_cast<int16_t>(br.extend(s) * q[z]);
        }
    }
    void block_dc(BitReader& br, Component& c, int16_t* d) {
        if (ah == 0) {
            const int t = br.decode(dc[c.td]);
            if (t > 15) jbad("bad DC magnitude");
            c.dc_pred += br.extend(t);
            d[0] = static_cast<int16_t>(c.dc_pred * (1 << al));
        } else if (br.bit()) {
            d[0] = static_cast<int16_t>(d[0] + (1 << al));
        }
    }
    void block_ac(BitReader& br, Component& c, int16_t* d) {
        if (ah == 0) {  // first AC scan (G.1.2.2)
            if (eob_run > 0) {
                --eob_run;
                return;
            }
            for (int k = ss; k <= se;) {
                const int rs = br.decode(ac[c.ta]), r = rs >> 4, s = rs & 15;
                if (s == 0) {
                    if (r < 15) {
                        eob_run = (1 << r) - 1 + (r ? br.bits(r) : 0);
                        break;
                    }
                    k += 16;
                    continue;
                }
                k += r;
                if (k > 63) jbad("AC coefficient past the block");
                d[kNatural[k++]] = static_cast<int16_t>(br.extend(s) * (1 << al));
            }
            return;
        }
        // refinement scan (G.1.2.3)
        const int16_t bit = static_cast<int16_t>(1 << al);
        auto refine = [&](int16_t& v) {
            if (br.bit() && (v & bit) == 0) v = static_cast<int16_t>(v > 0 ? v + bit : v - bit);
        };
        int k = ss;
        if (eob_run == 0) {
            while (k <= se) {
                const int rs = br.decode(ac[c.ta]);
                int r = rs >> 4;
                const int s = rs & 15;
                int16_t val = 0;
                if (s == 0) {
                    if (r < 15) {
                        eob_run = (1 << r) + (r ? br.bits(r) : 0);
                        break;  // the rest of the band is refined below
                    }
                } else {
                    if (s != 1) jbad("bad refinement magnitude");
                    val = br.bit() ? bit : static_cast<int16_t>(-bit);
                }
                // skip r zero-history coefficients (refining the nonzero ones met), then place val (if any)
                while (k <= se) {
                    int16_t& v = d[kNatural[k++]];
                    if (v != 0) {
                        refine(v);
                    } else {
                        if (r == 0) {
                            if (val) v = val;
                            break;
                        }
                        --r;
                    }
                }
            }
        }
        if (eob_run > 0) {
            for (; k <= se; ++k) {
                int16_t& v = d[kNatural[k]];
                if (v != 0) refine(v);
            }
            --eob_run;
        }
    }

    void scan() {
        BitReader br{p, end};
        for (int i = 0; i < ncomp; ++i) comp[i].dc_pred = 0;
        eob_run = 0;
        int todo = restart_interval ? restart_interval : -1;
        auto restart = [&]() {
            if (todo < 0 || --todo > 0) return;
            br.restart();
            for (int i = 0; i < ncomp; ++i) comp[i].dc_pred = 0;
            eob_run = 0;
            todo = restart_interval;
        };
        auto do_block = [&](Component& c, int bx, int by) {
            int16_t* d = block(c, bx, by);
            if (!progressive) block_sequential(br, c, d);
            else if (ss == 0) block_dc(br, c, d);
            else block_ac(br, c, d);
        };
        if (scan_n == 1) {  // non-interleaved: the component's own blocks in raster order
            Component& c = comp[order[0]];
            const int bw = (c.x + 7) / 8, bh = (c.y + 7) / 8;
            for (int by = 0; by < bh; ++by)
                for (int bx = 0; bx < bw; ++bx) {
                    do_block(c, bx, by);
                    if (!(by == bh - 1 && bx == bw - 1)) restart();
                }
        } else {
            for (int my = 0; my < mcuy; ++my)
                for (int mx = 0; mx < mcux; ++mx) {
                    for (int k = 0; k < scan_n; ++k) {
                        Component& c = comp[order[k]];
                        for (int y = 0; y < c.v; ++y)
                            for (int x = 0; x < c.h; ++x) do_block(c, mx * c.h + x, my * c.v + y);
                    }
                    if (!(my == mcuy - 1 && mx == mcux - 1)) restart();
                }
        }
        // continue after the entropy data: at the marker that ended it, or the next one in the stream
        p = br.p;
        pending = br.marker;
    }
    int pending = -1;

    DecodedImage decode() {
        if (end - p < 2 || p[0] != 0xFF || p[1] != 0xD8) jbad("no SOI marker");
        p += 2;
        bool have_frame = false;
        for (;;) {
            int m = pending >= 0 ? pending : next_marker();
            pending = -1;
            if (m < 0) {
                if (!have_frame) jbad("no frame");
                break;  // tolerate a missing EOI after the last scan
            }
            if (m == 0xD9) break;                                   // EOI
            if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7)) continue;     // stray SOI / RSTn
            if (m == 0xC0 || m == 0xC1 || m == 0xC2) {
                if (have_frame) jbad("second frame");
                frame(m);
                have_frame = true;
            } else if (m >= 0xC3 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
                jbad("unsupported coding process (lossless, hierarchical or arithmetic)");
            } else if (m == 0xC4) {
                dht();
            } else if (m == 0xDB) {
                dqt();
            } else if (m == 0xDD) {
                if (u16() != 4) jbad("bad DRI");
                restart_interval = u16();
            } else if (m == 0xDA) {
                if (!have_frame) jbad("scan before frame");
                scan_header();
                scan();
            } else if (m == 0xDC) {  // DNL
                if (u16() != 4) jbad("bad DNL");
                if (u16() != H) jbad("bad DNL height");
            } else if ((m >= 0xE0 && m <= 0xEF) || m == 0xFE) {
                app(m);
            } else {
                const int len = u16();  // any other marker segment: skip it
                if (len < 2 || end - p < len - 2) jbad("bad marker segment");
                p += len - 2;
            }
        }
        // inverse DCT of every block (progressive: after dequantizing with the final tables)
        for (int i = 0; i < ncomp; ++i) {
            Component& c = comp[i];
            const int bw = (c.x + 7) / 8, bh = (c.y + 7) / 8;
            for (int by = 0; by < bh; ++by)
                for (int bx = 0; bx < bw; ++bx) {
                    int16_t* d = block(c, bx, by);
                    if (progressive)
                        for (int k = 0; k < 64; ++k) d[k] = static_cast<int16_t>(d[k] * quant[c.tq][k]);
                    idct_block(d, c.plane.data() + static_cast<size_t>(by) * 8 * c.w2 + static_cast<size_t>(bx) * 8, c.w2);
                }
        }
        return to_pixels();
    }

    // upsampling (stb_image's resamplers: vertical/horizontal/both 2x triangle filters, nearest for other ratios)
    static void up_v2(uint8_t* out, const uint8_t* near, const uint8_t* far, int w) {
        for (int i = 0; i < w; ++i) out[i] = static_cast<uint8_t>((3 * near[i] + far[i] + 2) >> 2);
    }
    static void up_h2(uint8_t* out, const uint8_t* in, int w) {
        if (w == 1) {
            out[0] = out[1] = in[0];
            return;
        }
        out[0] = in[0];
        out[1] = static_cast<uint8_t>((in[0] * 3 + in[1] + 2) >> 2);
        int i = 1;
        for (; i < w - 1; ++i) {
            const int n = 3 * in[i] + 2;
            out[2 * i] = static_cast<uint8_t>((n + in[i - 1]) >> 2);
            out[2 * i + 1] = static_cast<uint8_t>((n + in[i + 1]) >> 2);
        }
        out[2 * i] = static_cast<uint8_t>((in[w - 2] * 3 + in[w - 1] + 2) >> 2);
        out[2 * i + 1] = in[w - 1];
    }
    static void up_hv2(uint8_t* out, const uint8_t* near, const uint8_t* far, int w) {
        if (w == 1) {
            out[0] = out[1] = static_cast<uint8_t>((3 * near[0] + far[0] + 2) >> 2);
            return;
        }
        int t1 = 3 * near[0] + far[0];
        out[0] = static_cast<uint8_t>((t1 + 2) >> 2);
        for (int i = 1; i < w; ++i) {
            const int t0 = t1;
            t1 = 3 * near[i] + far[i];
            out[2 * i - 1] = static_cast<uint8_t>((3 * t0 + t1 + 8) >> 4);
            out[2 * i] = static_cast<uint8_t>((3 * t1 + t0 + 8) >> 4);
        }
        out[2 * w - 1] = static_cast<uint8_t>((t1 + 2) >> 2);
    }

    DecodedImage to_pixels() {
        const bool is_rgb = ncomp == 3 && ((comp[0].id == 'R' && comp[1].id == 'G' && comp[2].id == 'B') || (adobe_transform == 0 && !jfif));
        DecodedImage img;
        img.w = W;
        img.h = H;
        img.channels = ncomp >= 3 ? 3 : 1;
        img.data.assign(static_cast<size_t>(W) * H * img.channels, 0);
        struct Rs {
            int hs, vs, ystep, ypos, wlo;
            const uint8_t *line0, *line1;
            std::vector<uint8_t> buf;
        } rs[4];
        for (int k = 0; k < ncomp; ++k) {
            rs[k].hs = hmax / comp[k].h;
            rs[k].vs = vmax / comp[k].v;
            rs[k].ystep = rs[k].vs >> 1;
            rs[k].ypos = 0;
            rs[k].wlo = (W + rs[k].hs - 1) / rs[k].hs;
            rs[k].line0 = rs[k].line1 = comp[k].plane.data();
            rs[k].buf.assign(static_cast<size_t>(W) + 3, 0);
        }
        const uint8_t* row[4];
        for (int y = 0; y < H; ++y) {
            for (int k = 0; k < ncomp; ++k) {
                Rs& r = rs[k];
                const bool bot = r.ystep >= (r.vs >> 1);
                const uint8_t* near = bot ? r.line1 : r.line0;
                const uint8_t* far = bot ? r.line0 : r.line1;
                if (r.hs == 1 && r.vs == 1) row[k] = near;
                else if (r.hs == 1 && r.vs == 2) up_v2(r.buf.data(), near, far, r.wlo), row[k] = r.buf.data();
                else if (r.hs == 2 && r.vs == 1) up_h2(r.buf.data(), near, r.wlo), row[k] = r.buf.data();
                else if (r.hs == 2 && r.vs == 2) up_hv2(r.buf.data(), near, far, r.wlo), row[k] = r.buf.data();
                else {
                    for (int i = 0; i < r.wlo; ++i)
                        for (int j = 0; j < r.hs; ++j) r.buf[static_cast<size_t>(i) * r.hs + j] = near[i];
                    row[k] = r.buf.data();
                }
                if (++r.ystep >= r.vs) {
                    r.ystep = 0;
                    r.line0 = r.line1;
                    if (++r.ypos < comp[k].y) r.line1 += comp[k].w2;
                }
            }
            uint8_t* out = img.data.data() + static_cast<size_t>(y) * W * img.channels;
            if (img.channels == 1) {
                std::memcpy(out, row[0], static_cast<size_t>(W));
                continue;
            }
            for (int i = 0; i < W; ++i, out += 3) {
                if (ncomp == 3 && is_rgb) {
                    out[0] = row[0][i];
                    out[1] = row[1][i];
                    out[2] = row[2][i];
                } else if (ncomp == 4 && adobe_transform == 0) {  // CMYK (Adobe inverted)
                    const int m = row[3][i];
                    auto blinn = [](int x, int yv) {
                        const unsigned t = static_cast<unsigned>(x * yv + 128);
                        return static_cast<uint8_t>((t + (t >> 8)) >> 8);
                    };
                    out[0] = blinn(row[0][i], m);
                    out[1] = blinn(row[1][i], m);
                    out[2] = blinn(row[2][i], m);
                } else {
                    // YCbCr -> RGB in stb_image's 20-bit fixed point (its scalar and SIMD paths agree on these values)
                    static const int kCr = static_cast<int>(1.40200f * 4096.0f + 0.5f) << 8, kCrG = static_cast<int>(0.71414f * 4096.0f + 0.5f) << 8,
                                     kCbG = static_cast<int>(0.34414f * 4096.0f + 0.5f) << 8, kCb = static_cast<int>(1.77200f * 4096.0f + 0.5f) << 8;
                    const int yf = (row[0][i] << 20) + (1 << 19);
                    const int cr = row[2][i] - 128, cb = row[1][i] - 128;
                    int r = yf + cr * kCr;
                    int g = yf + cr * -kCrG + static_cast<int>(static_cast<unsigned>(cb * -kCbG) & 0xffff0000u);
                    int b = yf + cb * kCb;
                    r >>= 20;
                    g >>= 20;
                    b >>= 20;
                    out[0] = clamp8(r);
                    out[1] = clamp8(g);
                    out[2] = clamp8(b);
                    if (ncomp == 4 && adobe_transform == 2) {  // YCCK
                        const int m = row[3][i];
                        auto blinn = [](int x, int yv) {
                            const unsigned t = static_cast<unsigned>(x * yv + 128);
                            return static_cast<uint8_t>((t + (t >> 8)) >> 8);
                        };
                        out[0] = blinn(255 - out[0], m);
                        out[1] = blinn(255 - out[1], m);
                        out[2] = blinn(255 - out[2], m);
                    }
                }
            }
        }
        return img;
    }
};

// ================================================================================================ PNG
[[noreturn]] void pbad(const std::string& what) { throw std::runtime_error("PNG: " + what); }
uint32_t be32(const uint8_t* p) { return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3]; }

int paeth(int a, int b, int c) {
    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    if (pa <= pb && pa <= pc) return a;
    return pb <= pc ? b : c;
}

}  // namespace

DecodedImage decode_jpeg(const uint8_t* bytes, size_t n) {
    Jpeg j(bytes, bytes + n);
    return j.decode();
}

DecodedImage decode_png(const uint8_t* b, size_t n) {
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (n < 8 || std::memcmp(b, sig, 8) != 0) pbad("bad signature");
    size_t at = 8;
    uint32_t W = 0, H = 0;
    int depth = 0, ctype = -1, interlace = 0;
    std::vector<uint8_t> idat, plte, trns;
    // tRNS as stb_image v2.27 takes it (stbi__parse_png_file), chunk by chunk: a palette image's tRNS sets the alpha of
    // its first entries (a later tRNS overwrites its own length of them; even an empty one makes the image 4-channel);
    // a gray / RGB image's tRNS is a colour key of one 16-bit sample per channel; refused after image data, before the
    // palette, or on a type with alpha
    std::vector<uint8_t> pal_alpha;
    bool pal_trns = false, key_trns = false;
    bool end_seen = false, first = true;
    while (at + 8 <= n && !end_seen) {
        const uint32_t len = be32(b + at);
        const uint8_t* type = b + at + 4;
        if (n - at < 12 || n - at - 12 < len) pbad("truncated chunk");  // length + type + data + CRC must all be present
        const uint8_t* d = b + at + 8;
        const bool ihdr = !std::memcmp(type, "IHDR", 4);
        if (first && !ihdr) pbad("first not IHDR");
        if (ihdr) {
            if (!first) pbad("multiple IHDR");
            if (len != 13) pbad("bad IHDR");
            W = be32(d);
            H = be32(d + 4);
            depth = d[8];
            ctype = d[9];
            if (d[10] != 0 || d[11] != 0) pbad("unknown compression or filter method");
            interlace = d[12];
            if (interlace > 1) pbad("bad interlace method");
        } else if (!std::memcmp(type, "PLTE", 4)) {
            if (len > 256 * 3 || len % 3) pbad("invalid PLTE");
            plte.assign(d, d + len);
            if (pal_alpha.size() < len / 3) pal_alpha.resize(len / 3, 255);
            std::fill(pal_alpha.begin(), pal_alpha.begin() + len / 3, static_cast<uint8_t>(255));
        } else if (!std::memcmp(type, "tRNS", 4)) {
            if (!idat.empty()) pbad("tRNS after IDAT");
            if (ctype == 3) {
                if (plte.empty()) pbad("tRNS before PLTE");
                if (len > plte.size() / 3) pbad("bad tRNS len");
                std::copy(d, d + len, pal_alpha.begin());
                pal_trns = true;
            } else {
                if (ctype == 4 || ctype == 6) pbad("tRNS with alpha");
                if (len != static_cast<uint32_t>(ctype == 2 ? 6 : 2)) pbad("bad tRNS len");
                trns.assign(d, d + len);
                key_trns = true;
            }
        } else if (!std::memcmp(type, "IDAT", 4)) {
            if (ctype == 3 && plte.empty()) pbad("no PLTE");
            idat.insert(idat.end(), d, d + len);
        } else if (!std::memcmp(type, "IEND", 4)) {
            end_seen = true;
        } else if (!(type[0] & 0x20)) {
            pbad(std::string("unknown critical chunk ") + std::string(reinterpret_cast<const char*>(type), 4));
        }
        at += 12 + len;
        first = false;
    }
    if (W == 0 || H == 0 || W > (1u << 24) || H > (1u << 24)) pbad("bad image size");
    int chans;
    switch (ctype) {
        case 0: chans = 1; break;
        case 2: chans = 3; break;
        case 3: chans = 1; break;
        case 4: chans = 2; break;
        case 6: chans = 4; break;
        default: pbad("bad color type");
    }
    const bool depth_ok = (ctype == 0 && (depth == 1 || depth == 2 || depth == 4 || depth == 8 || depth == 16)) ||
                          (ctype == 3 && (depth == 1 || depth == 2 || depth == 4 || depth == 8)) ||
                          ((ctype == 2 || ctype == 4 || ctype == 6) && (depth == 8 || depth == 16));
    if (!depth_ok) pbad("bad bit depth for the color type");
    if (ctype == 3 && (plte.empty() || plte.size() % 3)) pbad("missing or bad palette");
    // inflate
    std::vector<uint8_t> raw;
    {
        z_stream zs{};
        if (inflateInit(&zs) != Z_OK) pbad("zlib init");
        zs.next_in = idat.data();
        zs.avail_in = static_cast<uInt>(idat.size());
        uint8_t chunk[1 << 16];
        int rc;
        do {
            zs.next_out = chunk;
            zs.avail_out = sizeof chunk;
            rc = inflate(&zs, Z_NO_FLUSH);
            if (rc != Z_OK && rc != Z_STREAM_END) {
                inflateEnd(&zs);
                pbad("corrupt zlib data");
            }
            raw.insert(raw.end(), chunk, chunk + (sizeof chunk - zs.avail_out));
        } while (rc != Z_STREAM_END && (zs.avail_in > 0 || zs.avail_out == 0));
        inflateEnd(&zs);
    }
    const int bits_pp = chans * depth, bpp = std::max(1, bits_pp / 8);  // filter byte distance
    // samples (depth-expanded, 16-bit kept whole) of the full image, then the 8-bit result
    std::vector<uint16_t> samples(static_cast<size_t>(W) * H * chans);
    size_t pos = 0;
    auto pass = [&](uint32_t x0, uint32_t y0, uint32_t dx, uint32_t dy) {
        if (x0 >= W || y0 >= H) return;
        const uint32_t pw = (W - x0 + dx - 1) / dx, ph = (H - y0 + dy - 1) / dy;
        const size_t stride = (static_cast<size_t>(pw) * bits_pp + 7) / 8;
        std::vector<uint8_t> prev(stride, 0), cur(stride);
        for (uint32_t r = 0; r < ph; ++r) {
            if (pos + 1 + stride > raw.size()) pbad("truncated image data");
            const int f = raw[pos++];
            std::memcpy(cur.data(), raw.data() + pos, stride);
            pos += stride;
            for (size_t i = 0; i < stride; ++i) {
                const int a = i >= static_cast<size_t>(bpp) ? cur[i - bpp] : 0, up = prev[i], c = i >= static_cast<size_t>(bpp) ? prev[i - bpp] : 0;
                int v = cur[i];
                switch (f) {
                    case 0: break;
                    case 1: v += a; break;
                    case 2: v += up; break;
                    case 3: v += (a + up) >> 1; break;
                    case 4: v += paeth(a, up, c); break;
                    default: pbad("bad filter type");
                }
                cur[i] = static_cast<uint8_t>(v);
            }
            for (uint32_t x = 0; x < pw; ++x)
                for (int ch = 0; ch < chans; ++ch) {
                    const size_t sidx = static_cast<size_t>(x) * chans + ch;
                    uint16_t s;
                    if (depth == 16) s = static_cast<uint16_t>((cur[2 * sidx] << 8) | cur[2 * sidx + 1]);
                    else if (depth == 8) s = cur[sidx];
                    else {
                        const size_t bit = sidx * depth;
                        s = static_cast<uint16_t>((cur[bit / 8] >> (8 - depth - bit % 8)) & ((1 << depth) - 1));
                    }
                    samples[(static_cast<size_t>(y0 + r * dy) * W + x0 + x * dx) * chans + ch] = s;
                }
            std::swap(prev, cur);
        }
    };
    if (interlace) {
        static const uint32_t ax[7] = {0, 4, 0, 2, 0, 1, 0}, ay[7] = {0, 0, 4, 0, 2, 0, 1}, sx[7] = {8, 8, 4, 4, 2, 2, 1}, sy[7] = {8, 8, 8, 4, 4, 2, 2};
        for (int k = 0; k < 7; ++k) pass(ax[k], ay[k], sx[k], sy[k]);
    } else {
        pass(0, 0, 1, 1);
    }
    // to 8-bit channels, as stbi_load(..., 0): palette -> RGB (RGBA with tRNS), tRNS key -> an alpha channel
    DecodedImage img;
    img.w = static_cast<int>(W);
    img.h = static_cast<int>(H);
    const size_t npx = static_cast<size_t>(W) * H;
    if (ctype == 3) {
        const bool alpha = pal_trns;
        img.channels = alpha ? 4 : 3;
        img.data.resize(npx * img.channels);
        const size_t npal = plte.size() / 3;
        for (size_t i = 0; i < npx; ++i) {
            const size_t k = samples[i];
            if (k >= npal) pbad("palette index out of range");
            for (int c = 0; c < 3; ++c) img.data[i * img.channels + c] = plte[3 * k + c];
            if (alpha) img.data[i * 4 + 3] = pal_alpha[k];
        }
        return img;
    }
    const bool key = key_trns;
    img.channels = chans + (key ? 1 : 0);
    img.data.resize(npx * img.channels);
    static const int scale[9] = {0, 0xff, 0x55, 0, 0x11, 0, 0, 0, 0x01};
    // the colour key as stb compares it: 16-bit samples as they are; below 16 bits the key's low byte times the depth
    // scale, in 8 bits (stbi_uc), against the scaled 8-bit sample
    uint16_t kv[3] = {0, 0, 0};
    if (key)
        for (int c = 0; c < chans; ++c) {
            const uint16_t k16 = static_cast<uint16_t>((trns[2 * c] << 8) | trns[2 * c + 1]);
            kv[c] = depth == 16 ? k16 : static_cast<uint8_t>((k16 & 255) * scale[depth]);
        }
    for (size_t i = 0; i < npx; ++i) {
        bool transparent = key;
        for (int c = 0; c < chans; ++c) {
            const uint16_t s = samples[i * chans + c];
            const uint8_t v8 = depth == 16 ? static_cast<uint8_t>(s >> 8) : static_cast<uint8_t>(s * scale[depth]);
            if (key && (depth == 16 ? s : v8) != kv[c]) transparent = false;
            img.data[i * img.channels + c] = v8;
        }
        if (key) img.data[i * img.channels + chans] = transparent ? 0 : 255;
    }
    return img;
}

DecodedImage decode_image(const uint8_t* bytes, size_t n) {
    if (n >= 2 && bytes[0] == 0xFF && bytes[1] == 0xD8) return decode_jpeg(bytes, n);
    if (n >= 8 && bytes[0] == 137 && bytes[1] == 'P' && bytes[2] == 'N' && bytes[3] == 'G') return decode_png(bytes, n);
    throw std::runtime_error("unknown image format (JPEG and PNG are decoded)");
}

DecodedImage load_image_file(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open image " + path);
    const std::vector<uint8_t> bytes((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    try {
        return decode_image(bytes.data(), bytes.size());
    } catch (const std::exception& e) {
        throw std::runtime_error(path + ": " + e.what());
    }
}

}  // namespace art
