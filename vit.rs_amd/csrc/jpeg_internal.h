// jpeg_internal.h — the host half of the hybrid JPEG decoder (jpeg_host.cpp) shared with the
// device half (jpeg.hip).  SURVEY.md §8f-3: images are decoded for the train step's input
// (the reference's ViT::forward takes a prepared input array, /root/reference/train_vit.rs:188,
// encoder call :196).
//
// Split: the entropy decode (marker parsing, Huffman, DC prediction, restart intervals) is
// serial bit-level work and runs on host threads; everything per pixel — dequantisation, the
// 8x8 inverse DCT, chroma upsampling, YCbCr -> RGB, crop / resize / flip, normalisation — runs
// on the GPU.  Between the two, each 8x8 block travels as a 64-bit mask of its non-zero
// coefficients (zig-zag order, as decoded) plus those values (int16): ~4x fewer bytes over PCIe than the
// dense coefficients or the decoded pixels.
//
// Numerics follow the IJG libjpeg algorithms that libjpeg-turbo implements bit-exactly (the
// library Pillow links, used as the test oracle): jpeg_idct_islow (CONST_BITS 13, PASS1_BITS 2),
// the "fancy" triangle-filter chroma upsampling (h2v1, h2v2) and the fixed-point YCbCr -> RGB
// tables (SCALEBITS 16).  Baseline and extended sequential Huffman DCT, 8-bit, 1 or 3 components,
// chroma 4:4:4 / 4:2:2 / 4:2:0; progressive and arithmetic-coded files are rejected.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace vit {
namespace jpg {

constexpr int MAXC = 3;
enum Kind { GRAY = 0, YCC444 = 1, YCC422 = 2, YCC420 = 3 };

struct Frame {
    int w = 0, h = 0, nc = 0, kind = 0;
    int hs[MAXC]{}, vs[MAXC]{}, tq[MAXC]{}, id[MAXC]{};
    int hmax = 1, vmax = 1, mcux = 0, mcuy = 0;
    int bw[MAXC]{}, bh[MAXC]{};  // blocks per row / column of each component plane (MCU padded)
    int cw[MAXC]{}, ch[MAXC]{};  // valid samples of each component (ceil(w * hs / hmax), ...)
    uint16_t qt[MAXC][64]{};     // the component's quantisation table, natural order
    long long blocks() const {
        long long n = 0;
        for (int c = 0; c < nc; c++) n += (long long)bw[c] * bh[c];
        return n;
    }
};

// One image's blocks in sparse form, as decoded: masks[b] = bit k set <=> the coefficient at
// zig-zag position k of block b (component-major, each component's blocks row-major, bw x bh) is
// non-zero; its non-zero values, in zig-zag order, start at vals[voff[b]].
struct Sparse {
    std::vector<uint64_t> masks;
    std::vector<uint32_t> voff;
    std::vector<int16_t> vals;  // capacity; the first nvals are used
    long long nvals = 0;
};
// Parse the headers and entropy-decode every scan straight into the sparse form.  Returns false
// with a message on malformed / unsupported input.
bool decode_sparse(const uint8_t* data, size_t n, Frame& f, Sparse& sp, std::string& err);
// The same as dense int16 coefficients, natural order (tests: vit_jpeg_coefficients).
bool decode_coefficients(const uint8_t* data, size_t n, Frame& f, std::vector<int16_t>& coef, std::string& err);
// Headers only (dimensions, components, sampling kind).
bool parse_header(const uint8_t* data, size_t n, Frame& f, std::string& err);

}  // namespace jpg
}  // namespace vit
