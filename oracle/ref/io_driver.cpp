// io_driver — runs the reference's own image I/O for golden fixtures:
// image_io.cpp (compiled from /root/reference/source, with the vendored
// stb_image 2.28 / stb_image_write it includes) and the stbi_loadf call of
// Utils::read_image_float (utils.cpp:100-124; utils.cpp itself needs OIDN,
// which is absent, so its 20 lines are repeated here). Container-only.
//
//   io_driver hdr <in.hdr> <out.bin>   out: int32 w, h, then w*h RGBA f32 (alpha 0),
//                                      flipY = true (utils.h:16 default)
//   io_driver png <in.bin> <out.png>   in: int32 w, h, then w*h RGBA f32;
//                                      write_image_png(image, out) (image_io.cpp:165-182, flipY = true)
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "image.h"
#include "image_io.h"
#include "stb_image.h"

int main(int argc, char** argv)
{
    if (argc != 4) {
        std::fprintf(stderr, "usage: io_driver hdr|png <in> <out>\n");
        return 2;
    }
    const std::string cmd = argv[1];
    if (cmd == "hdr") {
        stbi_set_flip_vertically_on_load(true);  // utils.cpp:102
        int w = 0, h = 0, channels = 0;
        float* pixels = stbi_loadf(argv[2], &w, &h, &channels, 0);  // utils.cpp:105
        if (!pixels) return 1;
        Image output(w, h);
        for (int y = 0; y < h; y++)
            for (int x = 0; x < w; x++) {
                const int index = y * w + x;
                output[index] = Color(pixels[index * 3 + 0], pixels[index * 3 + 1], pixels[index * 3 + 2], 0.0f);
            }
        FILE* f = std::fopen(argv[3], "wb");
        if (!f) return 1;
        const int hdr[2] = {w, h};
        std::fwrite(hdr, 4, 2, f);
        for (int i = 0; i < w * h; i++) {
            const Color c = output[i];
            const float v[4] = {c.r, c.g, c.b, c.a};
            std::fwrite(v, 4, 4, f);
        }
        std::fclose(f);
        stbi_image_free(pixels);
        return 0;
    }
    if (cmd == "png") {
        FILE* f = std::fopen(argv[2], "rb");
        if (!f) return 1;
        int hdr[2];
        if (std::fread(hdr, 4, 2, f) != 2) return 1;
        Image img(hdr[0], hdr[1]);
        for (int i = 0; i < hdr[0] * hdr[1]; i++) {
            float v[4];
            if (std::fread(v, 4, 4, f) != 4) return 1;
            img[i] = Color(v[0], v[1], v[2], v[3]);
        }
        std::fclose(f);
        return write_image_png(img, argv[3]) ? 0 : 1;
    }
    return 2;
}
