// pt_checkpoint.cpp — checkpoint files of resumable frames (host side).
//
// The reference keeps nothing between runs: Renderer::render fills a frame in
// one go (src/renderer/mod.rs:67-114) and the GUI saves only the encoded
// image (src/bin/main.rs:281-289).  SURVEY §5 lists checkpoint / resume as the
// one auxiliary subsystem of the hot path: a long frame (4K x 4096 spp runs
// for seconds per GPU, minutes on the CPU) rendered in sample windows
// (pt_render_device_samples) can be stopped after any window and resumed from
// the per-pixel running sums, which these files hold.  Resuming is exact: the
// sums are f64 bit patterns and the next window adds its samples to them in
// sample order, as one launch over the whole frame would.
//
// Layout (little-endian): "PTCKPT01", the pt_checkpoint header (56 bytes),
// count doubles, and a 64-bit FNV-1a checksum over everything before it taken
// as 64-bit words (word-wise, so a 200 MB 4K frame checks at memory speed).
#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include <fcntl.h>
#include <unistd.h>

#include "../../include/rs_pathtracing.h"

static_assert(__BYTE_ORDER__ == __ORDER_LITTLE_ENDIAN__, "checkpoint files are written in host order");
static_assert(sizeof(pt_checkpoint) == 56, "pt_checkpoint is 56 bytes");

namespace {

constexpr char kMagic[8] = {'P', 'T', 'C', 'K', 'P', 'T', '0', '1'};
constexpr uint64_t kFnvOffset = 0xcbf29ce484222325ull, kFnvPrime = 0x100000001b3ull;
constexpr uint64_t kMaxCount = 1ull << 36;  // 512 GiB of sums: beyond any HBM shard

uint64_t fnv_words(uint64_t h, const void *p, size_t nwords) {
    const unsigned char *b = (const unsigned char *)p;
    for (size_t i = 0; i < nwords; i++) {
        uint64_t w;
        std::memcpy(&w, b + i * 8, 8);
        h = (h ^ w) * kFnvPrime;
    }
    return h;
}

// The sums a rank's d_out holds (pt_render_device's layout), or 0 for a header no frame has.
uint64_t expected_count(const pt_checkpoint &c) {
    if (c.width == 0 || c.height == 0 || c.samples_number == 0 || c.world == 0 || c.rank >= c.world) return 0;
    if (c.world == 1) return (uint64_t)c.width * c.height * 3;
    return (uint64_t)pt_shard_tiles(c.width, c.height, c.rank, c.world) * 256 * 3;
}

const char *header_problem(const pt_checkpoint &c) {
    if (c.width == 0 || c.height == 0 || c.samples_number == 0) return "empty frame";
    if (c.world == 0 || c.rank >= c.world) return "rank must be < world";
    if (c.samples_done > c.samples_number) return "samples_done > samples_number";
    if (c.reserved != 0) return "reserved field is not 0";
    if (c.count == 0 || c.count != expected_count(c) || c.count > kMaxCount)
        return "count does not match the frame's (rank's) pixels";
    return nullptr;
}

thread_local std::string g_ck_err;
std::atomic<unsigned long> g_tmp_seq{0};  // distinct temporaries for saves from several threads

}  // namespace

extern "C" {

// Defined in pt_api.cpp: the thread-local message pt_last_error returns.
__attribute__((visibility("hidden"))) void pt_set_last_error(const char *msg);

static int ck_fail(int code, const std::string &msg) {
    g_ck_err = msg;
    pt_set_last_error(g_ck_err.c_str());
    return code;
}

int pt_checkpoint_save(const char *path, const pt_checkpoint *c, const double *sums) {
    if (!path || !c || !sums) return ck_fail(PT_ERR_INVALID, "pt_checkpoint_save: null argument");
    if (const char *why = header_problem(*c)) return ck_fail(PT_ERR_INVALID, std::string("pt_checkpoint_save: ") + why);
    // a temporary next to the target, renamed over it once complete: a crash mid-write leaves the old file
    const std::string tmp = std::string(path) + ".tmp." + std::to_string((long)getpid()) + "." +
                            std::to_string(g_tmp_seq.fetch_add(1));
    FILE *f = std::fopen(tmp.c_str(), "wb");
    if (!f) return ck_fail(PT_ERR_IO, "pt_checkpoint_save: cannot open " + tmp + " for writing");
    uint64_t h = fnv_words(kFnvOffset, kMagic, 1);
    h = fnv_words(h, c, sizeof *c / 8);
    h = fnv_words(h, sums, c->count);
    bool ok = std::fwrite(kMagic, 1, 8, f) == 8 && std::fwrite(c, sizeof *c, 1, f) == 1 &&
              std::fwrite(sums, 8, c->count, f) == c->count && std::fwrite(&h, 8, 1, f) == 1;
    // durable before it replaces the target: the data reaches the disk before the rename, and the rename
    // (the directory entry) before the call returns, so a power loss leaves the old checkpoint or the new one
    ok = ok && std::fflush(f) == 0 && ::fsync(fileno(f)) == 0;
    ok = (std::fclose(f) == 0) && ok;
    if (!ok || std::rename(tmp.c_str(), path) != 0) {
        std::remove(tmp.c_str());
        return ck_fail(PT_ERR_IO, std::string("pt_checkpoint_save: short write to ") + path);
    }
    std::string dir(path);
    const size_t slash = dir.find_last_of('/');
    dir = slash == std::string::npos ? std::string(".") : (slash == 0 ? std::string("/") : dir.substr(0, slash));
    // The new file is in place from here on.  A file system that cannot sync a directory (EINVAL, ENOTSUP, e.g.
    // some FUSE and network mounts) makes the rename as durable as it can be: that is success.  Any other failure
    // is PT_ERR_IO, and the message says the checkpoint was written but its directory entry may not be durable.
    const int dfd = ::open(dir.c_str(), O_RDONLY | O_DIRECTORY);
    if (dfd < 0) return PT_OK;  // (no directory handle to sync: the rename itself has completed)
    const int rc = ::fsync(dfd);
    const int err = errno;
    ::close(dfd);
    if (rc != 0 && err != EINVAL && err != ENOTSUP && err != EOPNOTSUPP)
        return ck_fail(PT_ERR_IO, "pt_checkpoint_save: " + std::string(path) +
                                      " was written, but syncing its directory failed (the rename may not be durable)");
    return PT_OK;
}

int pt_checkpoint_load(const char *path, pt_checkpoint *c, double *sums, uint64_t capacity) {
    if (!path || !c) return ck_fail(PT_ERR_INVALID, "pt_checkpoint_load: null argument");
    FILE *f = std::fopen(path, "rb");
    if (!f) return ck_fail(PT_ERR_IO, std::string("pt_checkpoint_load: cannot open ") + path);
    struct Closer {
        FILE *f;
        ~Closer() { std::fclose(f); }
    } closer{f};
    char magic[8];
    pt_checkpoint hd;
    if (std::fread(magic, 1, 8, f) != 8 || std::memcmp(magic, kMagic, 8) != 0)
        return ck_fail(PT_ERR_IO, std::string("pt_checkpoint_load: ") + path + " is not a checkpoint file");
    if (std::fread(&hd, sizeof hd, 1, f) != 1)
        return ck_fail(PT_ERR_IO, std::string("pt_checkpoint_load: ") + path + " is truncated (header)");
    if (const char *why = header_problem(hd))
        return ck_fail(PT_ERR_IO, std::string("pt_checkpoint_load: ") + path + ": " + why);
    if (std::fseek(f, 0, SEEK_END) != 0)
        return ck_fail(PT_ERR_IO, std::string("pt_checkpoint_load: cannot seek in ") + path);
    const long size = std::ftell(f);
    const uint64_t want = 8 + sizeof hd + hd.count * 8 + 8;
    if (size < 0 || (uint64_t)size != want)
        return ck_fail(PT_ERR_IO, std::string("pt_checkpoint_load: ") + path + " has " + std::to_string(size) +
                                      " bytes, its header says " + std::to_string(want));
    if (sums) {
        if (capacity < hd.count)
            return ck_fail(PT_ERR_INVALID, "pt_checkpoint_load: sums holds " + std::to_string(capacity) +
                                               " doubles, the file " + std::to_string(hd.count));
        uint64_t stored = 0;
        if (std::fseek(f, (long)(8 + sizeof hd), SEEK_SET) != 0 || std::fread(sums, 8, hd.count, f) != hd.count ||
            std::fread(&stored, 8, 1, f) != 1)
            return ck_fail(PT_ERR_IO, std::string("pt_checkpoint_load: short read from ") + path);
        uint64_t h = fnv_words(kFnvOffset, kMagic, 1);
        h = fnv_words(h, &hd, sizeof hd / 8);
        h = fnv_words(h, sums, hd.count);
        if (h != stored) {
            std::memset(sums, 0, hd.count * 8);
            return ck_fail(PT_ERR_IO, std::string("pt_checkpoint_load: ") + path + " fails its checksum");
        }
    }
    *c = hd;
    return PT_OK;
}

}  // extern "C"
