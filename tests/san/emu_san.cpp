// TEST-ONLY sanitizer driver: the parallel entropy decoder's lane code
// (imagecodecs_amd/csrc/icx_spec_core.h through tests/emu/spec_emu.cpp, host-only build) under
// -fsanitize=address,undefined, run over every JPEG named on the command line with the sequential-
// chain emulator (emu_spec_decode) and the guess-write emulator (emu_gw_decode) at several lane
// sizes, leads and static-slot fractions. Exit status 0 = no sanitizer report.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../emu/spec_emu.cpp"

int main(int argc, char** argv) {
    const int64_t cap = 1 << 17;
    std::vector<int16_t> coef((size_t)cap * 64);
    std::vector<int32_t> dc(cap);
    int files = 0;
    for (int a = 1; a < argc; ++a) {
        FILE* f = std::fopen(argv[a], "rb");
        if (!f) return 2;
        std::vector<uint8_t> d;
        int c;
        while ((c = std::fgetc(f)) != EOF) d.push_back((uint8_t)c);
        std::fclose(f);
        int64_t nb = 0, st4[4] = {0, 0, 0, 0}, st8[8] = {0};
        int32_t status = 0;
        for (int sub : {64, 512, 2560}) {
            emu_spec_decode(d.data(), (int64_t)d.size(), sub, coef.data(), dc.data(), cap, &nb, &status, st4);
            emu_gw_decode(d.data(), (int64_t)d.size(), sub, sub == 64 ? 0 : 4096, sub == 512 ? 0.05 : 1.1, coef.data(),
                          dc.data(), cap, &nb, &status, st8);
        }
        ++files;
    }
    std::printf("sanitized %d files\n", files);
    return 0;
}
