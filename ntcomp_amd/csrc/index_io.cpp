// <prefix>.sbwt / <prefix>.lcs -- this library's native index files, the counterpart of
// kbo::index::serialize_sbwt (src/main.rs:138) and kbo::index::load_sbwt (src/main.rs:149,
// :190).  Like the reference, encode and decode both want the two files side by side
// (README.md:44).  The byte layout is this library's own (sbwt 0.3.11's serialisation is
// not available offline: DESIGN.md "Index files"); all integers little-endian:
//   .sbwt: "NTCSBWT1" u64 version=1, u64 n, u64 k, u64 C[4], u64 nwords, 4 x nwords u64
//   .lcs : "NTCLCS01" u64 n, n bytes
#include <cstdio>
#include <cstring>
#include <string>

#include "ntc_internal.h"

namespace ntc {

namespace {
struct File {
    FILE *f = nullptr;
    explicit File(const std::string &p, const char *mode) { f = std::fopen(p.c_str(), mode); }
    ~File() {
        if (f) std::fclose(f);
    }
};
bool wr(FILE *f, const void *p, size_t n) { return std::fwrite(p, 1, n, f) == n; }
bool rd(FILE *f, void *p, size_t n) { return std::fread(p, 1, n, f) == n; }
}  // namespace

bool save_index(const HostIndex &ix, const std::string &prefix, std::string &err) {
    const uint64_t nw = (ix.n + 63) / 64;
    {
        File f(prefix + ".sbwt", "wb");
        if (!f.f) { err = "cannot open " + prefix + ".sbwt for writing"; return false; }
        uint64_t hdr[1 + 1 + 1 + 4 + 1] = {1, ix.n, ix.k, ix.C[0], ix.C[1], ix.C[2], ix.C[3], nw};
        bool ok = wr(f.f, "NTCSBWT1", 8) && wr(f.f, hdr, sizeof(hdr));
        for (int c = 0; c < 4 && ok; c++) ok = wr(f.f, ix.rows[c].data(), nw * 8);
        if (!ok) { err = "write failed: " + prefix + ".sbwt"; return false; }
    }
    {
        File f(prefix + ".lcs", "wb");
        if (!f.f) { err = "cannot open " + prefix + ".lcs for writing"; return false; }
        uint64_t n = ix.n;
        if (!(wr(f.f, "NTCLCS01", 8) && wr(f.f, &n, 8) && wr(f.f, ix.lcs.data(), ix.n))) {
            err = "write failed: " + prefix + ".lcs";
            return false;
        }
    }
    return true;
}

bool load_index(const std::string &prefix, HostIndex &ix, std::string &err) {
    {
        File f(prefix + ".sbwt", "rb");
        if (!f.f) { err = "cannot open " + prefix + ".sbwt"; return false; }
        char magic[8];
        uint64_t hdr[8];
        if (!rd(f.f, magic, 8) || std::memcmp(magic, "NTCSBWT1", 8) != 0 || !rd(f.f, hdr, sizeof(hdr)) ||
            hdr[0] != 1) {
            err = prefix + ".sbwt: not an ntcomp-mi355x index (or an unsupported version)";
            return false;
        }
        ix.n = hdr[1];
        ix.k = (uint32_t)hdr[2];
        for (int c = 0; c < 4; c++) ix.C[c] = hdr[3 + c];
        uint64_t nw = hdr[7];
        if (nw != (ix.n + 63) / 64 || ix.k < 1 || ix.k > 255) {
            err = prefix + ".sbwt: inconsistent header";
            return false;
        }
        for (int c = 0; c < 4; c++) {
            ix.rows[c].assign(nw, 0);
            if (!rd(f.f, ix.rows[c].data(), nw * 8)) { err = prefix + ".sbwt: truncated"; return false; }
        }
    }
    {
        File f(prefix + ".lcs", "rb");
        if (!f.f) { err = "cannot open " + prefix + ".lcs"; return false; }
        char magic[8];
        uint64_t n = 0;
        if (!rd(f.f, magic, 8) || std::memcmp(magic, "NTCLCS01", 8) != 0 || !rd(f.f, &n, 8) || n != ix.n) {
            err = prefix + ".lcs: missing, foreign or not matching " + prefix + ".sbwt";
            return false;
        }
        ix.lcs.assign(n, 0);
        if (!rd(f.f, ix.lcs.data(), n)) { err = prefix + ".lcs: truncated"; return false; }
    }
    return true;
}

}  // namespace ntc
