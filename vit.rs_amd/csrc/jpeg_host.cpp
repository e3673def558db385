// jpeg_host.cpp — host entropy decoder of the hybrid JPEG path (jpeg_internal.h): JFIF/JPEG
// marker parsing and sequential Huffman decoding (ITU-T T.81 Annex F.2) into quantised DCT
// coefficients.  No pixel work happens here: the GPU (jpeg.hip) dequantises, transforms,
// upsamples, converts colour and resizes.
#include <cstring>

#include "jpeg_internal.h"

namespace vit {
namespace jpg {
namespace {

// zig-zag scan position -> natural (row-major) index
constexpr uint8_t kZig[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                              12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                              35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                              58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

constexpr int FAST = 11;  // look-up bits of the fast Huffman table
constexpr long long kMaxFramePixels = 1LL << 28;  // 16384 x 16384: larger headers are rejected

struct Huff {
    bool present = false;
    uint8_t fast_len[1 << FAST]{};  // 0: code longer than FAST bits
    uint8_t fast_sym[1 << FAST]{};
    int maxcode[18]{};               // largest code of each length (-1: none); [17] sentinel
    int valptr[17]{}, mincode[17]{};
    uint8_t vals[256]{};
    // AC tables: the whole (run, value) of a short code + its value bits in one look-up:
    // fast_ac[look] = value << 16 | run << 8 | bits consumed, 0 when the pair does not fit in FAST
    int32_t fast_ac[1 << FAST]{};

    void build_fast_ac() {
        for (int look = 0; look < (1 << FAST); look++) {
            fast_ac[look] = 0;
            const int l = fast_len[look];
            if (!l) continue;
            const int rs = fast_sym[look], r = rs >> 4, sz = rs & 15;
            if (!sz || l + sz > FAST) continue;
            int v = (look >> (FAST - l - sz)) & ((1 << sz) - 1);
            if (v < (1 << (sz - 1))) v -= (1 << sz) - 1;
            fast_ac[look] = (int32_t)((uint32_t)v << 16) | (r << 8) | (l + sz);
        }
    }

    bool build(const uint8_t* counts, const uint8_t* symbols, int nsym) {
        int code = 0, k = 0;
        memset(fast_len, 0, sizeof(fast_len));
        for (int len = 1; len <= 16; len++) {
            valptr[len] = k;
            mincode[len] = code;
            for (int i = 0; i < counts[len - 1]; i++, k++, code++) {
                if (code >= (1 << len)) return false;  // over-subscribed table
                if (len <= FAST) {
                    const int base = code << (FAST - len);
                    for (int j = 0; j < (1 << (FAST - len)); j++) {
                        fast_len[base + j] = (uint8_t)len;
                        fast_sym[base + j] = symbols[k];
                    }
                }
            }
            maxcode[len] = counts[len - 1] ? code - 1 : -1;
            code <<= 1;
        }
        maxcode[17] = 0x7fffffff;
        if (k != nsym) return false;
        memcpy(vals, symbols, (size_t)nsym);
        build_fast_ac();
        present = true;
        return true;
    }
};

// MSB-first bit reader over entropy-coded data: removes the 0xFF00 stuffing, stops at a marker
// (then supplies zero bits, as decoders do for truncated data)
struct Bits {
    const uint8_t* p;
    const uint8_t* end;
    uint64_t buf = 0;
    int cnt = 0;
    bool at_marker = false;

    void fill() {
        // fast path: 8 bytes without an 0xFF (no stuffing, no marker) append whole
        if (!at_marker && p + 8 <= end) {
            uint64_t w;
            memcpy(&w, p, 8);
            w = __builtin_bswap64(w);
            const uint64_t x = ~w;
            if (!((x - 0x0101010101010101ULL) & ~x & 0x8080808080808080ULL)) {
                const int nb = (64 - cnt) >> 3;
                buf |= (w >> (64 - 8 * nb)) << (64 - cnt - 8 * nb);
                p += nb;
                cnt += 8 * nb;
                return;
            }
        }
        while (cnt <= 56) {
            uint32_t b = 0;
            if (!at_marker && p < end) {
                b = *p;
                if (b == 0xFF) {
                    const uint8_t nx = p + 1 < end ? p[1] : 0xD9;
                    if (nx == 0x00) {
                        p += 2;
                    } else {
                        at_marker = true;
                        b = 0;
                    }
                } else {
                    p++;
                }
            }
            buf |= (uint64_t)b << (56 - cnt);
            cnt += 8;
        }
    }
    int get(int n) {  // 1 <= n <= 16
        if (cnt < n) fill();
        const int v = (int)(buf >> (64 - n));
        buf <<= n;
        cnt -= n;
        return v;
    }
    int decode(const Huff& h) {
        if (cnt < 16) fill();
        const int look = (int)(buf >> (64 - FAST));
        if (h.fast_len[look]) {
            const int l = h.fast_len[look];
            buf <<= l;
            cnt -= l;
            return h.fast_sym[look];
        }
        int l = FAST + 1;
        int code = (int)(buf >> (64 - l));
        while (l <= 16 && code > h.maxcode[l]) {
            l++;
            code = (int)(buf >> (64 - l));
        }
        if (l > 16) return -1;
        buf <<= l;
        cnt -= l;
        return h.vals[h.valptr[l] + code - h.mincode[l]];
    }
    // restart: drop the partial byte, consume the RSTn marker (searching forward if the reader
    // stopped short of it)
    bool restart(int expect) {
        buf = 0;
        cnt = 0;
        if (!at_marker) {
            while (p + 1 < end && !(p[0] == 0xFF && p[1] != 0x00 && p[1] != 0xFF)) p++;
        }
        at_marker = false;
        if (p + 1 < end && p[0] == 0xFF && p[1] == 0xD0 + expect) {
            p += 2;
            return true;
        }
        return false;
    }
};

inline int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

inline int be16(const uint8_t* q) { return (q[0] << 8) | q[1]; }

struct Parser {
    const uint8_t* d;
    size_t n;
    Frame& f;
    std::string& err;
    uint16_t qt[4][64]{};
    bool qt_present[4]{};
    Huff dc[4], ac[4];
    int restart_interval = 0;
    bool have_frame = false;

    bool fail(const char* m) {
        err = m;
        return false;
    }

    bool frame(const uint8_t* q, int len) {
        // a second SOF would resize the frame under scan state sized by the first (libjpeg
        // rejects it too)
        if (have_frame) return fail("duplicate SOF marker");
        if (len < 8) return fail("SOF segment too short");
        if (q[0] != 8) return fail("only 8-bit samples are supported");
        f.h = be16(q + 1);
        f.w = be16(q + 3);
        f.nc = q[5];
        if (f.w <= 0 || f.h <= 0) return fail("zero image dimension (DNL not supported)");
        // host allocations (masks, offsets, values) scale with the header's pixel count: bound it
        // before any entropy data is read
        if ((long long)f.w * f.h > kMaxFramePixels) return fail("image too large (more than 2^28 pixels)");
        if (f.nc != 1 && f.nc != 3) return fail("only 1- or 3-component images are supported");
        if (len < 6 + 3 * f.nc) return fail("SOF segment too short");
        f.hmax = f.vmax = 1;
        for (int c = 0; c < f.nc; c++) {
            f.id[c] = q[6 + 3 * c];
            f.hs[c] = q[7 + 3 * c] >> 4;
            f.vs[c] = q[7 + 3 * c] & 15;
            f.tq[c] = q[8 + 3 * c];
            if (f.hs[c] < 1 || f.hs[c] > 4 || f.vs[c] < 1 || f.vs[c] > 4 || f.tq[c] > 3)
                return fail("bad component parameters");
            f.hmax = f.hs[c] > f.hmax ? f.hs[c] : f.hmax;
            f.vmax = f.vs[c] > f.vmax ? f.vs[c] : f.vmax;
        }
        if (f.nc == 1) {  // a single-component image is one block per MCU whatever its factors
            f.hs[0] = f.vs[0] = f.hmax = f.vmax = 1;
            f.kind = GRAY;
        } else {
            const int rh1 = f.hmax / f.hs[1], rv1 = f.vmax / f.vs[1];
            const bool chroma_same = f.hs[1] == f.hs[2] && f.vs[1] == f.vs[2];
            const bool luma_full = f.hs[0] == f.hmax && f.vs[0] == f.vmax;
            const bool exact = f.hmax % f.hs[1] == 0 && f.vmax % f.vs[1] == 0;
            if (!chroma_same || !luma_full || !exact) return fail("unsupported chroma sampling");
            if (rh1 == 1 && rv1 == 1) f.kind = YCC444;
            else if (rh1 == 2 && rv1 == 1) f.kind = YCC422;
            else if (rh1 == 2 && rv1 == 2) f.kind = YCC420;
            else return fail("unsupported chroma sampling");
        }
        f.mcux = (f.w + 8 * f.hmax - 1) / (8 * f.hmax);
        f.mcuy = (f.h + 8 * f.vmax - 1) / (8 * f.vmax);
        for (int c = 0; c < f.nc; c++) {
            f.bw[c] = f.mcux * f.hs[c];
            f.bh[c] = f.mcuy * f.vs[c];
            f.cw[c] = (f.w * f.hs[c] + f.hmax - 1) / f.hmax;
            f.ch[c] = (f.h * f.vs[c] + f.vmax - 1) / f.vmax;
        }
        have_frame = true;
        return true;
    }

    bool dqt(const uint8_t* q, int len) {
        int o = 0;
        while (o < len) {
            const int pq = q[o] >> 4, t = q[o] & 15;
            if (t > 3 || pq > 1) return fail("bad DQT");
            const int need = 1 + 64 * (pq + 1);
            if (o + need > len) return fail("DQT segment too short");
            for (int k = 0; k < 64; k++)
                qt[t][kZig[k]] = pq ? (uint16_t)be16(q + o + 1 + 2 * k) : q[o + 1 + k];
            qt_present[t] = true;
            o += need;
        }
        return true;
    }

    bool dht(const uint8_t* q, int len) {
        int o = 0;
        while (o < len) {
            if (o + 17 > len) return fail("DHT segment too short");
            const int tc = q[o] >> 4, th = q[o] & 15;
            if (tc > 1 || th > 3) return fail("bad DHT");
            int nsym = 0;
            for (int i = 0; i < 16; i++) nsym += q[o + 1 + i];
            if (nsym > 256 || o + 17 + nsym > len) return fail("bad DHT symbol count");
            Huff& h = tc ? ac[th] : dc[th];
            if (!h.build(q + o + 1, q + o + 17, nsym)) return fail("bad Huffman table");
            o += 17 + nsym;
        }
        return true;
    }

    // one block straight into the sparse form: the non-zero coefficients in zig-zag order at out,
    // their zig-zag positions as the bits of m; returns the count (or -1).  The bit buffer lives
    // in locals for the block (written back around refills).
    int block(Bits& bits, const Huff& hd, const Huff& ha, int& pred, int16_t* out, uint64_t& m) {
        uint64_t buf = bits.buf;
        int cnt = bits.cnt;
        auto refill = [&]() {
            bits.buf = buf;
            bits.cnt = cnt;
            bits.fill();
            buf = bits.buf;
            cnt = bits.cnt;
        };
        auto huff = [&](const Huff& h) -> int {
            if (cnt < 16) refill();
            const int look = (int)(buf >> (64 - FAST));
            if (h.fast_len[look]) {
                const int l = h.fast_len[look];
                buf <<= l;
                cnt -= l;
                return h.fast_sym[look];
            }
            int l = FAST + 1;
            int code = (int)(buf >> (64 - l));
            while (l <= 16 && code > h.maxcode[l]) {
                l++;
                code = (int)(buf >> (64 - l));
            }
            if (l > 16) return -1;
            buf <<= l;
            cnt -= l;
            return h.vals[h.valptr[l] + code - h.mincode[l]];
        };
        auto bitsn = [&](int n) -> int {  // 1 <= n <= 16
            if (cnt < n) refill();
            const int v = (int)(buf >> (64 - n));
            buf <<= n;
            cnt -= n;
            return v;
        };
        const int s = huff(hd);
        if (s < 0 || s > 11) return fail("bad DC code") ? 0 : -1;
        pred += s ? extend(bitsn(s), s) : 0;
        int n = 0;
        uint64_t mm = 0;
        if (pred) {
            mm = 1;
            out[n++] = (int16_t)pred;
        }
        for (int k = 1; k < 64;) {
            if (cnt < 16) refill();
            const int32_t fa = ha.fast_ac[buf >> (64 - FAST)];
            if (fa) {  // run + value in one look-up
                const int l = fa & 255;
                k += (fa >> 8) & 255;
                buf <<= l;
                cnt -= l;
                if (k > 63) return fail("AC coefficient index past 63") ? 0 : -1;
                mm |= 1ULL << k;
                out[n++] = (int16_t)(fa >> 16);
                k++;
                continue;
            }
            const int rs = huff(ha);
            if (rs < 0) return fail("bad AC code") ? 0 : -1;
            const int r = rs >> 4, sz = rs & 15;
            if (sz) {
                k += r;
                if (k > 63) return fail("AC coefficient index past 63") ? 0 : -1;
                mm |= 1ULL << k;
                out[n++] = (int16_t)extend(bitsn(sz), sz);
                k++;
            } else {
                if (r != 15) break;  // EOB
                k += 16;
            }
        }
        bits.buf = buf;
        bits.cnt = cnt;
        m = mm;
        return n;
    }
    // block bi (component-major index) of the image into the sink
    bool emit(Bits& b, const Huff& hd, const Huff& ha, int& pred, long long bi, Sparse& sp) {
        if (sp.vals.size() < (size_t)sp.nvals + 64) sp.vals.resize(sp.vals.size() * 2 + 64 * 64);
        uint64_t m;
        const int cnt = block(b, hd, ha, pred, sp.vals.data() + sp.nvals, m);
        if (cnt < 0) return false;
        sp.masks[(size_t)bi] = m;
        sp.voff[(size_t)bi] = (uint32_t)sp.nvals;
        sp.nvals += cnt;
        return true;
    }

    // one scan; returns the position after its entropy-coded data
    bool scan(const uint8_t* q, int len, const uint8_t*& pos, Sparse& sp) {
        if (!have_frame) return fail("SOS before SOF");
        const int ns = q[0];
        if (ns < 1 || ns > f.nc || len < 4 + 2 * ns) return fail("bad SOS");
        int comp[MAXC], td[MAXC], ta[MAXC];
        for (int i = 0; i < ns; i++) {
            const int cid = q[1 + 2 * i];
            comp[i] = -1;
            for (int c = 0; c < f.nc; c++)
                if (f.id[c] == cid) comp[i] = c;
            if (comp[i] < 0) return fail("SOS names an unknown component");
            td[i] = q[2 + 2 * i] >> 4;
            ta[i] = q[2 + 2 * i] & 15;
            if (td[i] > 3 || ta[i] > 3 || !dc[td[i]].present || !ac[ta[i]].present)
                return fail("SOS uses a missing Huffman table");
        }
        const int ss = q[1 + 2 * ns], se = q[2 + 2 * ns], ahl = q[3 + 2 * ns];
        if (ss != 0 || se != 63 || ahl != 0) return fail("not a sequential DCT scan");
        long long base[MAXC];  // first block of each component
        long long o = 0;
        for (int c = 0; c < f.nc; c++) {
            base[c] = o;
            o += (long long)f.bw[c] * f.bh[c];
        }
        Bits b{pos, d + n};
        int pred[MAXC] = {0, 0, 0};
        int mcus_left = restart_interval, rst = 0;
        auto do_restart = [&]() -> bool {
            if (!b.restart(rst)) return fail("missing restart marker");
            rst = (rst + 1) & 7;
            pred[0] = pred[1] = pred[2] = 0;
            mcus_left = restart_interval;
            return true;
        };
        if (ns == 1) {  // non-interleaved: the component's own block grid, one block per MCU
            const int c = comp[0];
            const int nbx = (f.cw[c] + 7) / 8, nby = (f.ch[c] + 7) / 8;
            for (int by = 0; by < nby; by++)
                for (int bx = 0; bx < nbx; bx++) {
                    if (restart_interval && mcus_left == 0 && !do_restart()) return false;
                    if (!emit(b, dc[td[0]], ac[ta[0]], pred[0], base[c] + (long long)by * f.bw[c] + bx, sp))
                        return false;
                    mcus_left--;
                }
        } else {
            for (int my = 0; my < f.mcuy; my++)
                for (int mx = 0; mx < f.mcux; mx++) {
                    if (restart_interval && mcus_left == 0 && !do_restart()) return false;
                    for (int i = 0; i < ns; i++) {
                        const int c = comp[i];
                        for (int v = 0; v < f.vs[c]; v++)
                            for (int h = 0; h < f.hs[c]; h++) {
                                const long long bi = (long long)(my * f.vs[c] + v) * f.bw[c] + mx * f.hs[c] + h;
                                if (!emit(b, dc[td[i]], ac[ta[i]], pred[i], base[c] + bi, sp)) return false;
                            }
                    }
                    mcus_left--;
                }
        }
        // resume marker parsing at the next marker after the entropy-coded data
        const uint8_t* e = b.p;
        while (e + 1 < d + n && !(e[0] == 0xFF && e[1] != 0x00 && !(e[1] >= 0xD0 && e[1] <= 0xD7))) e++;
        pos = e;
        return true;
    }

    bool run(Sparse* sp) {
        if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) return fail("not a JPEG file (no SOI)");
        const uint8_t* p = d + 2;
        const uint8_t* end = d + n;
        bool scanned = false;
        while (p + 1 < end) {
            if (p[0] != 0xFF) {
                p++;
                continue;
            }
            const int m = p[1];
            p += 2;
            if (m == 0xFF || m == 0x01 || (m >= 0xD0 && m <= 0xD7)) {
                if (m == 0xFF) p--;  // fill byte
                continue;
            }
            if (m == 0xD9) break;  // EOI
            if (p + 2 > end) return fail("truncated marker segment");
            const int len = be16(p) - 2;
            const uint8_t* q = p + 2;
            if (len < 0 || q + len > end) return fail("truncated marker segment");
            switch (m) {
                case 0xC0: case 0xC1:
                    if (!frame(q, len)) return false;
                    if (!sp) return true;  // headers only
                    break;
                case 0xC2: case 0xC6: case 0xCA: case 0xCE: return fail("progressive JPEG is not supported");
                case 0xC3: case 0xC5: case 0xC7: case 0xCB: case 0xCD: case 0xCF:
                    return fail("lossless / hierarchical JPEG is not supported");
                case 0xC9: return fail("arithmetic-coded JPEG is not supported");
                case 0xC4: if (!dht(q, len)) return false; break;
                case 0xDB: if (!dqt(q, len)) return false; break;
                case 0xDD:
                    if (len < 2) return fail("bad DRI");
                    restart_interval = be16(q);
                    break;
                case 0xDA: {
                    if (!have_frame) return fail("SOS before SOF");
                    if (!sp) return true;
                    if (!scanned) {
                        for (int c = 0; c < f.nc; c++) {
                            if (!qt_present[f.tq[c]]) return fail("missing quantisation table");
                            memcpy(f.qt[c], qt[f.tq[c]], sizeof(f.qt[c]));
                        }
                        // blocks no scan codes (padding of non-interleaved scans) stay all-zero
                        sp->masks.assign((size_t)f.blocks(), 0);
                        sp->voff.assign((size_t)f.blocks(), 0);
                        if (sp->vals.size() < (size_t)f.blocks() * 8) sp->vals.resize((size_t)f.blocks() * 8);
                        sp->nvals = 0;
                        scanned = true;
                    }
                    const uint8_t* pos = q + len;
                    if (!scan(q, len, pos, *sp)) return false;
                    p = pos;
                    continue;
                }
                default: break;  // APPn, COM, DNL, ...: skipped
            }
            p = q + len;
        }
        if (!have_frame) return fail("no SOF marker");
        if (sp && !scanned) return fail("no scan");
        return true;
    }
};

}  // namespace

bool parse_header(const uint8_t* data, size_t n, Frame& f, std::string& err) {
    Parser ps{data, n, f, err};
    return ps.run(nullptr);
}

bool decode_sparse(const uint8_t* data, size_t n, Frame& f, Sparse& sp, std::string& err) {
    Parser ps{data, n, f, err};
    return ps.run(&sp);
}

bool decode_coefficients(const uint8_t* data, size_t n, Frame& f, std::vector<int16_t>& coef, std::string& err) {
    Sparse sp;
    if (!decode_sparse(data, n, f, sp, err)) return false;
    const long long nb = f.blocks();
    coef.assign((size_t)nb * 64, 0);
    for (long long b = 0; b < nb; b++) {
        uint64_t m = sp.masks[(size_t)b];
        const int16_t* v = sp.vals.data() + sp.voff[(size_t)b];
        while (m) {
            const int k = __builtin_ctzll(m);
            coef[(size_t)b * 64 + kZig[k]] = *v++;
            m &= m - 1;
        }
    }
    return true;
}

}  // namespace jpg
}  // namespace vit
