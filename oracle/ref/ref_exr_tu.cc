/*
 * TEST INFRASTRUCTURE ONLY -- never linked into the product (imagecodecs_amd).
 *
 * Implementation translation unit for the reference's tinyexr, compiled IN PLACE from
 * /root/reference/tinyexr.h (nothing is copied). The reference builds it with miniz
 * (codecs.cpp:27-29), which it does not vendor. tinyexr's own documented alternative is used
 * instead: TINYEXR_USE_MINIZ 0 with "your own zlib-compatible API header" included first
 * (tinyexr.h:109-112, 664-671), here the system zlib. mz_uncompress and zlib's uncompress take
 * the same arguments and both check the zlib header and the Adler-32 (RFC 1950/1951), so a valid
 * ZIP/ZIPS chunk inflates to the same bytes; NONE / RLE / PIZ chunks and all header and offset
 * logic do not touch the inflate library at all.
 * Build: oracle/Makefile target `ref` -> oracle/_ref/libref_exr.so (gitignored, container only).
 *
 * The exports add no arithmetic: a buffer-in / buffer-out surface for ctypes.
 */
#include <malloc.h>
#include <zlib.h>

#include <cstdlib>
#include <cstring>

#define TINYEXR_USE_MINIZ 0
#define TINYEXR_IMPLEMENTATION
#include "tinyexr.h"

extern "C" {

/* glibc's M_PERTURB: malloc'd memory is filled with a pattern byte, and allocations stay on the
 * heap (no zero-filled mmap), so two runs with different bytes show which output floats
 * tinyexr never wrote (uninitialised rows / tiles). */
void ref_exr_perturb(int byte) {
    mallopt(M_MMAP_THRESHOLD, 32 * 1024 * 1024);
    mallopt(M_PERTURB, byte);
}

/* Image::readExr (codecs.cpp:464-493): LoadEXRFromMemory over the bytes given (the caller
 * appends the trailing 0xFF the reference's ifstream loop adds, :468-471). Returns tinyexr's
 * code; on success *w, *h are set and min(w*h*4, cap) floats are copied to `out`. */
int ref_exr_load(const unsigned char* mem, long long size, float* out, long long cap, int* w, int* h) {
    float* rgba = nullptr;
    const char* err = nullptr;
    *w = 0;
    *h = 0;
    const int ret = LoadEXRFromMemory(&rgba, w, h, mem, (size_t)size, &err);
    if (err) FreeEXRErrorMessage(err);
    if (ret == TINYEXR_SUCCESS && rgba) {
        const long long n = (long long)(*w) * (long long)(*h) * 4;
        std::memcpy(out, rgba, (size_t)((n < cap ? n : cap) * (long long)sizeof(float)));
        std::free(rgba);
    }
    return ret;
}
}
