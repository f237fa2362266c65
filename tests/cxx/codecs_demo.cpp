// Drop-in check for include/imagecodecs/codecs.h: the reference's Image::read/write usage,
// unchanged, against libicx.so.
//   codecs_demo errors            -- unknown extension / missing GPU behaviour (no GPU needed)
//   codecs_demo read IN OUT.rgb   -- decode IN, dump w h d + raw pixels to OUT.rgb
//   codecs_demo roundtrip IN OUT.jpg -- decode IN, write OUT.jpg (tje quality 3)
#include <cstdio>
#include <cstring>
#include <stdexcept>

#include "imagecodecs/codecs.h"

int main(int argc, char** argv) {
    if (argc >= 2 && !std::strcmp(argv[1], "errors")) {
        ImageCodecs::Image img;
        try {
            img.read("x.webp");
            return 1;
        } catch (const std::invalid_argument&) {
            std::puts("invalid_argument ok");
        }
        try {
            img.write("x.bmp");
            return 1;
        } catch (const std::invalid_argument&) {
            std::puts("invalid_argument ok");
        }
        try {
            img.read(argc >= 3 ? argv[2] : "missing.jpg");
            std::puts("read ok");
        } catch (const std::runtime_error& e) {
            std::printf("runtime_error: %s\n", e.what());
        }
        return 0;
    }
    if (argc == 4 && !std::strcmp(argv[1], "read")) {
        ImageCodecs::Image img;
        img.read(argv[2]);
        std::FILE* f = std::fopen(argv[3], "wb");
        int hdr[3] = {img.cols(), img.rows(), img.channels()};
        std::fwrite(hdr, sizeof hdr, 1, f);
        std::fwrite(*img.data(), 1, img.totalBytes(), f);
        std::fclose(f);
        std::printf("%d %d %d\n", img.cols(), img.rows(), img.channels());
        return 0;
    }
    if (argc == 4 && !std::strcmp(argv[1], "roundtrip")) {
        ImageCodecs::Image img;
        img.read(argv[2]);
        img.write(argv[3]);
        std::printf("write %s\n", img.lastWriteOk() ? "ok" : "failed");
        return img.lastWriteOk() ? 0 : 1;
    }
    std::fprintf(stderr, "usage: codecs_demo errors|read IN OUT|roundtrip IN OUT\n");
    return 2;
}
