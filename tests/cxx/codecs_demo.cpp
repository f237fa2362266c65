// Drop-in check for include/imagecodecs/codecs.h: the reference's Image::read/write usage,
// unchanged, against libicx.so.
//   codecs_demo errors            -- unknown extension / missing GPU behaviour (no GPU needed)
//   codecs_demo read IN OUT.rgb   -- decode IN, dump w h d + raw pixels to OUT.rgb
//   codecs_demo roundtrip IN OUT.jpg -- decode IN, write OUT.jpg (tje quality 3)
//   codecs_demo utils IN OUT       -- decode IN, then dump the pixels after flip(), after
//                                     swapBR() as well, and idx<T>() of a few elements
//   codecs_demo loadutils OUT      -- the same on a load()-ed 5x3x4 byte buffer (no GPU)
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
    if ((argc == 4 && !std::strcmp(argv[1], "utils")) || (argc == 3 && !std::strcmp(argv[1], "loadutils"))) {
        ImageCodecs::Image img;
        const bool loaded = argc == 3;
        if (loaded) {
            unsigned char* px = new unsigned char[5 * 3 * 4];
            for (int k = 0; k < 60; ++k) px[k] = (unsigned char)(k * 7 + 3);
            img.load(px, 5, 3, 4);  // adopted: ~Image delete[]s it
        } else {
            img.read(argv[2]);
        }
        std::FILE* f = std::fopen(argv[loaded ? 2 : 3], "wb");
        int hdr[4] = {img.cols(), img.rows(), img.channels(), img.byteSize()};
        std::fwrite(hdr, sizeof hdr, 1, f);
        img.flip();
        std::fwrite(*img.data(), 1, img.totalBytes(), f);
        img.swapBR();
        std::fwrite(*img.data(), 1, img.totalBytes(), f);
        const int pts[3][3] = {{0, 0, 0}, {img.rows() - 1, img.cols() - 1, img.channels() - 1}, {img.rows() / 2, 1, 1}};
        for (auto& p : pts) {
            if (img.type() == ImageCodecs::Type::FLOAT) {
                const float v = img.idx<float>(p[0], p[1], p[2]);
                std::fwrite(&v, sizeof v, 1, f);
            } else {
                const unsigned char v = img.idx<unsigned char>(p[0], p[1], p[2]);
                std::fwrite(&v, 1, 1, f);
            }
        }
        std::fclose(f);
        std::printf("%d %d %d\n", img.cols(), img.rows(), img.channels());
        return 0;
    }
    std::fprintf(stderr, "usage: codecs_demo errors|read IN OUT|roundtrip IN OUT|utils IN OUT|loadutils OUT\n");
    return 2;
}
