// pt_image.cpp — image output of the display-encoded frame (host side).
//
// The reference saves the GUI's RGBA8 frame with image::save_buffer(...,
// ColorType::Rgba8) to images/rendered.png (src/bin/main.rs:71-82,
// main_raylib.rs:64-74).  pt_write_png writes the same pixels as a PNG
// (RGBA, 8 bit, no interlace) whose zlib stream uses stored (uncompressed)
// deflate blocks: any PNG reader decodes it to exactly these bytes.
// pt_write_ppm writes binary PPM (P6, alpha dropped) for quick viewing.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rs_pathtracing.h"

namespace {

struct CrcTable {
    uint32_t t[256];
    CrcTable() {
        for (uint32_t n = 0; n < 256; n++) {
            uint32_t c = n;
            for (int k = 0; k < 8; k++) c = (c & 1u) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
            t[n] = c;
        }
    }
};

// built once, on first use, by whichever thread gets there first (a function-local static's initialisation is
// thread-safe): pt_write_png may be called from several host threads at once
const uint32_t *crc_table() {
    static const CrcTable table;
    return table.t;
}

uint32_t crc32(const uint8_t *p, size_t n, uint32_t c = 0xFFFFFFFFu) {
    const uint32_t *tab = crc_table();
    for (size_t i = 0; i < n; i++) c = tab[(c ^ p[i]) & 0xFFu] ^ (c >> 8);
    return c;
}

void be32(std::vector<uint8_t> &o, uint32_t v) {
    o.push_back((uint8_t)(v >> 24));
    o.push_back((uint8_t)(v >> 16));
    o.push_back((uint8_t)(v >> 8));
    o.push_back((uint8_t)v);
}

void chunk(std::vector<uint8_t> &o, const char *type, const std::vector<uint8_t> &data) {
    be32(o, (uint32_t)data.size());
    const size_t at = o.size();
    o.insert(o.end(), type, type + 4);
    o.insert(o.end(), data.begin(), data.end());
    be32(o, crc32(o.data() + at, 4 + data.size()) ^ 0xFFFFFFFFu);
}

int write_file(const char *path, const std::vector<uint8_t> &bytes, std::string *err) {
    FILE *f = std::fopen(path, "wb");
    if (!f) {
        *err = std::string("cannot open ") + path + " for writing";
        return PT_ERR_INVALID;
    }
    const size_t n = std::fwrite(bytes.data(), 1, bytes.size(), f);
    const int closed = std::fclose(f);
    if (n != bytes.size() || closed != 0) {
        *err = std::string("short write to ") + path;
        return PT_ERR_INVALID;
    }
    return PT_OK;
}

thread_local std::string g_img_err;

}  // namespace

extern "C" {

// Defined in pt_api.cpp: the thread-local message pt_last_error returns.
__attribute__((visibility("hidden"))) void pt_set_last_error(const char *msg);


int pt_write_png(const char *path, const uint8_t *rgba, uint32_t width, uint32_t height) {
    if (!path || !rgba || width == 0 || height == 0) {
        pt_set_last_error("pt_write_png: null argument or empty image");
        return PT_ERR_INVALID;
    }
    // a PNG chunk's length is a 32-bit field (and < 2^31 by the spec): the one IDAT chunk must fit
    const size_t row = (size_t)width * 4;
    const size_t raw_bytes = (row + 1) * height;
    if (raw_bytes + raw_bytes / 65535 * 5 + 64 >= ((size_t)1 << 31)) {
        pt_set_last_error("pt_write_png: image too large for one IDAT chunk");
        return PT_ERR_INVALID;
    }
    std::vector<uint8_t> png = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
    std::vector<uint8_t> ihdr;
    be32(ihdr, width);
    be32(ihdr, height);
    ihdr.insert(ihdr.end(), {8, 6, 0, 0, 0});  // 8 bit, RGBA, deflate, filter method 0, no interlace
    chunk(png, "IHDR", ihdr);
    // raw scanlines: filter type 0 (None) then the row's RGBA bytes
    std::vector<uint8_t> raw;
    raw.reserve(raw_bytes);
    for (uint32_t y = 0; y < height; y++) {
        raw.push_back(0);
        raw.insert(raw.end(), rgba + (size_t)y * row, rgba + (size_t)(y + 1) * row);
    }
    // zlib: CMF/FLG (deflate, 32K window, no dictionary, check bits), stored
    // blocks of <= 65535 bytes, Adler-32 of the raw data
    std::vector<uint8_t> z = {0x78, 0x01};
    size_t pos = 0;
    do {
        const size_t n = raw.size() - pos < 65535 ? raw.size() - pos : 65535;
        const bool last = pos + n == raw.size();
        z.push_back(last ? 1 : 0);
        z.push_back((uint8_t)(n & 0xFF));
        z.push_back((uint8_t)(n >> 8));
        z.push_back((uint8_t)(~n & 0xFF));
        z.push_back((uint8_t)((~n >> 8) & 0xFF));
        z.insert(z.end(), raw.begin() + pos, raw.begin() + pos + n);
        pos += n;
    } while (pos < raw.size());
    uint32_t a = 1, b = 0;
    for (uint8_t v : raw) {
        a = (a + v) % 65521u;
        b = (b + a) % 65521u;
    }
    be32(z, (b << 16) | a);
    chunk(png, "IDAT", z);
    chunk(png, "IEND", {});
    int rc = write_file(path, png, &g_img_err);
    if (rc) pt_set_last_error(g_img_err.c_str());
    return rc;
}

int pt_write_ppm(const char *path, const uint8_t *rgba, uint32_t width, uint32_t height) {
    if (!path || !rgba || width == 0 || height == 0) {
        pt_set_last_error("pt_write_ppm: null argument or empty image");
        return PT_ERR_INVALID;
    }
    char head[64];
    const int hn = std::snprintf(head, sizeof head, "P6\n%u %u\n255\n", width, height);
    std::vector<uint8_t> out(head, head + hn);
    out.reserve(out.size() + (size_t)width * height * 3);
    for (size_t i = 0; i < (size_t)width * height; i++) out.insert(out.end(), rgba + i * 4, rgba + i * 4 + 3);
    int rc = write_file(path, out, &g_img_err);
    if (rc) pt_set_last_error(g_img_err.c_str());
    return rc;
}

}  // extern "C"
