// sanitize_host.cpp -- the host mirror's device-free code (mesh readers, `.inst` parsing) under
// AddressSanitizer + UndefinedBehaviorSanitizer (csrc/Makefile `sanitize`, run by
// tests/test_sanitize_cpu.py).  Usage: sanitize_host <mesh or .inst file>...
// For every mesh file it also feeds truncated and byte-flipped copies to the reader, which
// must report an error or return triangles, never read out of bounds.
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "instance_file_map.hpp"
#include "mesh_loader.hpp"

static std::string slurp(const std::string &p) {
    std::ifstream f(p, std::ios::binary);
    std::ostringstream s;
    s << f.rdbuf();
    return s.str();
}

static void spit(const std::string &p, const std::string &data) {
    std::ofstream f(p, std::ios::binary);
    f << data;
}

static double checksum(const std::vector<double> &t) {
    double s = 0;
    for (size_t i = 0; i < t.size(); ++i) s += t[i] * (double)((i % 7) + 1);
    return s;
}

int main(int argc, char **argv) {
    int bad = 0;
    for (int a = 1; a < argc; ++a) {
        const std::string path = argv[a];
        const std::string ext = path.size() > 5 ? path.substr(path.size() - 5) : path;
        if (ext == ".inst") {
            mpt_host::InstanceFileMap m(path);
            const bool ok = m.exists("Agent Type") && !m.value("Agent Type").empty();
            std::printf("%s: Agent Type %s\n", path.c_str(), ok ? m.value("Agent Type").c_str() : "?");
            bad += ok ? 0 : 1;
            continue;
        }
        const mpt_host::MeshFile m = mpt_host::load_mesh(path);
        const std::vector<double> soup = m.soup(), last = m.last_nonempty();
        std::printf("%s: %zu submeshes, %zu / %zu triangles, checksum %.6f%s\n", path.c_str(), m.submeshes.size(),
                    soup.size() / 9, last.size() / 9, checksum(soup), m.error ? " (error)" : "");
        bad += m.error ? 1 : 0;
        // damaged copies: truncated at several lengths, and bytes flipped
        const std::string data = slurp(path);
        const std::string dot = path.substr(path.find_last_of('.'));
        const std::string tmp = std::string("/tmp/mpt_sanitize_case") + dot;
        for (int k = 1; k <= 8; ++k) {
            spit(tmp, data.substr(0, data.size() * k / 9));
            (void)mpt_host::load_mesh(tmp).soup();
            std::string flipped = data;
            for (size_t i = (size_t)k * 131; i < flipped.size(); i += 997) flipped[i] = (char)(flipped[i] ^ (0x5a + k));
            spit(tmp, flipped);
            (void)mpt_host::load_mesh(tmp).soup();
        }
        std::remove(tmp.c_str());
    }
    std::printf("sanitize_host %s\n", bad ? "FAILED" : "ok");
    return bad ? 1 : 0;
}
