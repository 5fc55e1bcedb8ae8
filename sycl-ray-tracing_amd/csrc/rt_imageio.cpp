// rt_imageio.cpp — the reference's image input and output stages, host side.
//
//  * read_hdr: Utils::read_image_float (utils.cpp:100-124) on a Radiance .hdr
//    file, i.e. stb_image 2.28's stbi__hdr_load (stb_image.h:7086-7286,
//    vendored in the reference) with req_comp 3 and the vertical flip of
//    stbi_set_flip_vertically_on_load(true). Decoding is exact: a texel is
//    (float)m * 2^(e - 136) (stbi__hdr_convert :7130-7155), a product that is
//    always representable, so the floats match stb_image's bit for bit
//    (tests/test_imageio.py against fixtures made by the reference's code).
//  * rgba8 / write_png: write_image_png (image_io.cpp:165-182): x * 255,
//    clamp to [0, 255] with image_io.cpp's clamp (NaN passes through), float
//    -> unsigned char as g++ on x86-64 converts it (cvttss2si, low byte), then
//    flipY and PNG. stb_image_write's deflate is not reproduced: the file is
//    a valid PNG with stored (uncompressed) deflate blocks whose decoded
//    pixels equal the reference's.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rt_fp.h"
#include "rt_scene.h"

namespace rt {
namespace {

// stbi__context over a whole file: get8 returns 0 past the end (stbi__get8).
struct Bytes {
    std::vector<unsigned char> d;
    size_t p = 0;
    bool eof() const { return p >= d.size(); }
    int get8() { return p < d.size() ? d[p++] : 0; }
};

// stbi__hdr_gettoken (:7108-7128)
std::string gettoken(Bytes& z)
{
    std::string s;
    char c = (char)z.get8();
    while (!z.eof() && c != '\n') {
        s.push_back(c);
        if (s.size() == 1023) {
            while (!z.eof() && z.get8() != '\n') {
            }
            break;
        }
        c = (char)z.get8();
    }
    return s;
}

// stbi__hdr_convert (:7130-7155), req_comp 3
void convert(float* out, const unsigned char* in)
{
    if (in[3] != 0) {
        const float f1 = (float)std::ldexp(1.0f, in[3] - (int)(128 + 8));
        out[0] = in[0] * f1;
        out[1] = in[1] * f1;
        out[2] = in[2] * f1;
    } else {
        out[0] = out[1] = out[2] = 0;
    }
}

}  // namespace

int read_hdr(const char* path, bool flip_y, int& width, int& height, std::vector<float>& rgb, std::string& err)
{
    Bytes s;
    {
        FILE* f = std::fopen(path, "rb");
        if (!f) {
            err = std::string("cannot open ") + path;
            return -1;
        }
        unsigned char buf[1 << 16];
        size_t n;
        while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) s.d.insert(s.d.end(), buf, buf + n);
        std::fclose(f);
    }
    const std::string head = gettoken(s);
    if (head != "#?RADIANCE" && head != "#?RGBE") {
        err = "not HDR";
        return -1;
    }
    bool valid = false;
    for (;;) {
        const std::string t = gettoken(s);
        if (t.empty()) break;
        if (t == "FORMAT=32-bit_rle_rgbe") valid = true;
    }
    if (!valid) {
        err = "unsupported HDR format";
        return -1;
    }
    std::string t = gettoken(s);
    if (t.compare(0, 3, "-Y ") != 0) {
        err = "unsupported HDR data layout";
        return -1;
    }
    const char* tok = t.c_str() + 3;
    char* endp = nullptr;
    const int h = (int)std::strtol(tok, &endp, 10);
    tok = endp;
    while (*tok == ' ') ++tok;
    if (std::strncmp(tok, "+X ", 3) != 0) {
        err = "unsupported HDR data layout";
        return -1;
    }
    const int w = (int)std::strtol(tok + 3, nullptr, 10);
    if (h > (1 << 24) || w > (1 << 24) || w <= 0 || h <= 0) {
        err = "bad HDR dimensions";
        return -1;
    }
    width = w;
    height = h;
    rgb.assign((size_t)w * h * 3, 0.0f);
    float* data = rgb.data();
    int i = 0, j = 0;
    bool flat = w < 8 || w >= 32768;
    if (!flat) {
        std::vector<unsigned char> scan((size_t)w * 4);
        for (j = 0; j < h; ++j) {
            const int c1 = s.get8(), c2 = s.get8();
            int len = s.get8();
            if (c1 != 2 || c2 != 2 || (len & 0x80)) {
                // not run-length encoded: this is a pixel of flat data, and the
                // reference restarts the flat loop at (j = 0, i = 1) (:7229-7242)
                const unsigned char rgbe[4] = {(unsigned char)c1, (unsigned char)c2, (unsigned char)len,
                                               (unsigned char)s.get8()};
                convert(data, rgbe);
                i = 1;
                j = 0;
                flat = true;
                break;
            }
            len <<= 8;
            len |= s.get8();
            if (len != w) {
                err = "invalid decoded scanline length";
                return -1;
            }
            for (int k = 0; k < 4; ++k) {
                int x = 0, nleft;
                while ((nleft = w - x) > 0) {
                    int count = s.get8();
                    if (count > 128) {
                        const int value = s.get8();
                        count -= 128;
                        if (count == 0 || count > nleft) {
                            err = "bad RLE data in HDR";
                            return -1;
                        }
                        for (int z = 0; z < count; ++z) scan[(size_t)x++ * 4 + k] = (unsigned char)value;
                    } else {
                        if (count == 0 || count > nleft) {
                            err = "bad RLE data in HDR";
                            return -1;
                        }
                        for (int z = 0; z < count; ++z) scan[(size_t)x++ * 4 + k] = (unsigned char)s.get8();
                    }
                }
            }
            for (int x = 0; x < w; ++x) convert(data + ((size_t)j * w + x) * 3, &scan[(size_t)x * 4]);
        }
        if (!flat) i = w;  // (RLE completed: nothing left for the flat loop)
    }
    if (flat) {
        for (; j < h; ++j, i = 0)
            for (; i < w; ++i) {
                unsigned char rgbe[4];
                for (int c = 0; c < 4; c++) rgbe[c] = (unsigned char)s.get8();
                convert(data + ((size_t)j * w + i) * 3, rgbe);
            }
    }
    if (flip_y)  // stbi__vertical_flip (:1220-1243)
        for (int y = 0; y < h / 2; y++)
            for (size_t k = 0; k < (size_t)w * 3; k++)
                std::swap(rgb[(size_t)y * w * 3 + k], rgb[(size_t)(h - 1 - y) * w * 3 + k]);
    return 0;
}

// write_image_png's conversion loop (image_io.cpp:165-177).
void rgba8(const float* rgba, size_t n_px, unsigned char* out)
{
    auto clamp = [](float x, float mn, float mx) {  // image_io.cpp:156-161
        if (x < mn) return mn;
        if (x > mx) return mx;
        return x;
    };
    for (size_t i = 0; i < 4 * n_px; i++) out[i] = (unsigned char)rt_f2i(clamp(rgba[i] * 255, 0, 255));
}

namespace {
uint32_t crc32(const unsigned char* p, size_t n, uint32_t c = 0)
{
    c = ~c;
    for (size_t i = 0; i < n; i++) {
        c ^= p[i];
        for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    }
    return ~c;
}
void put32(std::vector<unsigned char>& v, uint32_t x)
{
    for (int s = 24; s >= 0; s -= 8) v.push_back((unsigned char)(x >> s));
}
void chunk(std::vector<unsigned char>& png, const char* type, const std::vector<unsigned char>& data)
{
    put32(png, (uint32_t)data.size());
    const size_t at = png.size();
    png.insert(png.end(), type, type + 4);
    png.insert(png.end(), data.begin(), data.end());
    put32(png, crc32(&png[at], data.size() + 4));
}
}  // namespace

int write_png(const char* path, const float* rgba, int w, int h, bool flip_y, std::string& err)
{
    if (w <= 0 || h <= 0) {
        err = "empty image";  // write_image_png returns false for image.size() == 0
        return -1;
    }
    std::vector<unsigned char> px((size_t)w * h * 4);
    rgba8(rgba, (size_t)w * h, px.data());
    // raw scanlines (filter 0), flipped like stbi_flip_vertically_on_write
    std::vector<unsigned char> raw;
    raw.reserve((size_t)h * (4 * (size_t)w + 1));
    for (int y = 0; y < h; y++) {
        const int sy = flip_y ? h - 1 - y : y;
        raw.push_back(0);
        raw.insert(raw.end(), px.begin() + (size_t)sy * w * 4, px.begin() + (size_t)(sy + 1) * w * 4);
    }
    // zlib stream of stored deflate blocks
    std::vector<unsigned char> z = {0x78, 0x01};
    size_t off = 0;
    do {
        const size_t n = std::min<size_t>(65535, raw.size() - off);
        const bool last = off + n == raw.size();
        z.push_back(last ? 1 : 0);
        z.push_back((unsigned char)(n & 0xff));
        z.push_back((unsigned char)(n >> 8));
        z.push_back((unsigned char)(~n & 0xff));
        z.push_back((unsigned char)((~n >> 8) & 0xff));
        z.insert(z.end(), raw.begin() + off, raw.begin() + off + n);
        off += n;
    } while (off < raw.size());
    uint32_t a = 1, b = 0;
    for (unsigned char c : raw) {
        a = (a + c) % 65521u;
        b = (b + a) % 65521u;
    }
    put32(z, (b << 16) | a);
    std::vector<unsigned char> png = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    std::vector<unsigned char> ihdr;
    put32(ihdr, (uint32_t)w);
    put32(ihdr, (uint32_t)h);
    ihdr.insert(ihdr.end(), {8, 6, 0, 0, 0});  // 8-bit RGBA, deflate, filter 0, no interlace
    chunk(png, "IHDR", ihdr);
    chunk(png, "IDAT", z);
    chunk(png, "IEND", {});
    FILE* f = std::fopen(path, "wb");
    if (!f) {
        err = std::string("cannot write ") + path;
        return -1;
    }
    const bool ok = std::fwrite(png.data(), 1, png.size(), f) == png.size();
    std::fclose(f);
    if (!ok) err = "short write";
    return ok ? 0 : -1;
}

}  // namespace rt
