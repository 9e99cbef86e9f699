// mesh_loader.cpp -- see mesh_loader.hpp.
#include "mesh_loader.hpp"

#include <algorithm>
#include <cctype>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>

namespace mpt_host {

std::vector<double> MeshFile::soup() const {
    std::vector<double> out;
    for (const auto &s : submeshes) out.insert(out.end(), s.tris.begin(), s.tris.end());
    return out;
}

std::vector<double> MeshFile::last_nonempty() const {
    for (auto it = submeshes.rbegin(); it != submeshes.rend(); ++it)
        if (!it->tris.empty()) return it->tris;
    return {};
}

namespace {

bool read_file(const std::string &path, std::string &out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::ostringstream ss;
    ss << f.rdbuf();
    out = ss.str();
    return true;
}

std::string lower_ext(const std::string &path) {
    const auto p = path.find_last_of('.');
    std::string e = p == std::string::npos ? "" : path.substr(p + 1);
    for (auto &c : e) c = (char)std::tolower((unsigned char)c);
    return e;
}

double f32(const char *s, char **end) { return (double)std::strtof(s, end); }

// ------------------------------------------------------------------ OBJ
MeshFile load_obj(const std::string &text) {
    MeshFile m;
    std::vector<double> verts;
    SubMesh cur;
    bool have_cur = false;
    std::istringstream in(text);
    std::string line;
    auto flush = [&]() {
        if (have_cur) m.submeshes.push_back(std::move(cur));
        cur = SubMesh();
        have_cur = false;
    };
    while (std::getline(in, line)) {
        if (line.empty() || line[0] == '#') continue;
        std::istringstream ls(line);
        std::string tag;
        ls >> tag;
        if (tag == "o" || tag == "g") {
            flush();
            std::string rest;
            std::getline(ls, rest);
            cur.name = rest;
            have_cur = true;
        } else if (tag == "v") {
            std::string a, b, c;
            ls >> a >> b >> c;
            verts.push_back(f32(a.c_str(), nullptr));
            verts.push_back(f32(b.c_str(), nullptr));
            verts.push_back(f32(c.c_str(), nullptr));
        } else if (tag == "f") {
            std::vector<long> idx;
            std::string tok;
            while (ls >> tok) idx.push_back(std::strtol(tok.c_str(), nullptr, 10));
            if (idx.size() != 3) continue;  // non-triangle faces are skipped
            have_cur = true;
            for (long i : idx) {
                const long v = i > 0 ? i - 1 : (long)(verts.size() / 3) + i;
                if (v < 0 || (size_t)(3 * v + 2) >= verts.size()) {
                    m.error = true;
                    m.message = "obj: face index out of range";
                    return m;
                }
                cur.tris.insert(cur.tris.end(), verts.begin() + 3 * v, verts.begin() + 3 * v + 3);
            }
        }
    }
    flush();
    return m;
}

// ------------------------------------------------------------------ COLLADA (minimal XML walk)
struct XNode {
    std::string tag;
    std::map<std::string, std::string> attr;
    std::string text;
    std::vector<XNode> kids;
    const XNode *child(const std::string &t) const {
        for (const auto &k : kids)
            if (k.tag == t) return &k;
        return nullptr;
    }
};

struct XParser {
    const std::string &s;
    size_t i = 0;
    explicit XParser(const std::string &src) : s(src) {}
    void skip_ws() {
        while (i < s.size() && std::isspace((unsigned char)s[i])) ++i;
    }
    // parse children until </closing>
    void parse_children(XNode &parent) {
        while (i < s.size()) {
            const size_t lt = s.find('<', i);
            if (lt == std::string::npos) {
                parent.text += s.substr(i);
                i = s.size();
                return;
            }
            parent.text += s.substr(i, lt - i);
            i = lt;
            if (s.compare(i, 4, "<!--") == 0) {
                const size_t e = s.find("-->", i);
                i = e == std::string::npos ? s.size() : e + 3;
                continue;
            }
            if (s.compare(i, 2, "<?") == 0 || s.compare(i, 2, "<!") == 0) {
                const size_t e = s.find('>', i);
                i = e == std::string::npos ? s.size() : e + 1;
                continue;
            }
            if (s.compare(i, 2, "</") == 0) {
                const size_t e = s.find('>', i);
                i = e == std::string::npos ? s.size() : e + 1;
                return;
            }
            XNode n;
            ++i;
            size_t st = i;
            while (i < s.size() && !std::isspace((unsigned char)s[i]) && s[i] != '>' && s[i] != '/') ++i;
            n.tag = s.substr(st, i - st);
            bool selfclose = false;
            for (;;) {
                skip_ws();
                if (i >= s.size()) break;
                if (s[i] == '/') {
                    selfclose = true;
                    ++i;
                    continue;
                }
                if (s[i] == '>') {
                    ++i;
                    break;
                }
                st = i;
                while (i < s.size() && s[i] != '=' && !std::isspace((unsigned char)s[i])) ++i;
                std::string key = s.substr(st, i - st);
                skip_ws();
                if (i < s.size() && s[i] == '=') ++i;
                skip_ws();
                if (i < s.size() && (s[i] == '"' || s[i] == '\'')) {
                    const char q = s[i++];
                    st = i;
                    while (i < s.size() && s[i] != q) ++i;
                    n.attr[key] = s.substr(st, i - st);
                    ++i;
                }
            }
            if (!selfclose) parse_children(n);
            parent.kids.push_back(std::move(n));
        }
    }
};

void collect(const XNode &n, const std::string &tag, std::vector<const XNode *> &out) {
    if (n.tag == tag) out.push_back(&n);
    for (const auto &k : n.kids) collect(k, tag, out);
}

std::vector<long> parse_ints(const std::string &t) {
    std::vector<long> v;
    const char *p = t.c_str();
    char *e = nullptr;
    for (;;) {
        while (*p && std::isspace((unsigned char)*p)) ++p;
        if (!*p) break;
        const long x = std::strtol(p, &e, 10);
        if (e == p) break;
        v.push_back(x);
        p = e;
    }
    return v;
}

std::vector<double> parse_floats(const std::string &t) {
    std::vector<double> v;
    const char *p = t.c_str();
    char *e = nullptr;
    for (;;) {
        while (*p && std::isspace((unsigned char)*p)) ++p;
        if (!*p) break;
        const double x = f32(p, &e);
        if (e == p) break;
        v.push_back(x);
        p = e;
    }
    return v;
}

std::string strip_hash(const std::string &s) { return !s.empty() && s[0] == '#' ? s.substr(1) : s; }

MeshFile load_dae(const std::string &text) {
    MeshFile m;
    XNode root;
    XParser(text).parse_children(root);
    std::vector<const XNode *> geoms;
    collect(root, "library_geometries", geoms);
    std::map<std::string, std::vector<double>> sources;
    std::vector<const XNode *> srcs;
    collect(root, "source", srcs);
    for (const XNode *s : srcs) {
        const XNode *fa = s->child("float_array");
        if (fa) sources[s->attr.count("id") ? s->attr.at("id") : ""] = parse_floats(fa->text);
    }
    for (const XNode *lib : geoms)
        for (const auto &g : lib->kids) {
            if (g.tag != "geometry") continue;
            const XNode *mesh = g.child("mesh");
            if (!mesh) continue;
            std::map<std::string, std::string> vmap;  // <vertices id> -> POSITION source
            for (const auto &k : mesh->kids)
                if (k.tag == "vertices")
                    for (const auto &in : k.kids)
                        if (in.tag == "input" && in.attr.count("semantic") && in.attr.at("semantic") == "POSITION")
                            vmap[k.attr.count("id") ? k.attr.at("id") : ""] = strip_hash(in.attr.at("source"));
            for (const auto &prim : mesh->kids) {
                if (prim.tag != "triangles" && prim.tag != "polylist") continue;
                int stride = 1, voff = -1;
                std::string vsrc;
                for (const auto &in : prim.kids) {
                    if (in.tag != "input") continue;
                    const int off = in.attr.count("offset") ? std::atoi(in.attr.at("offset").c_str()) : 0;
                    stride = std::max(stride, off + 1);
                    if (in.attr.count("semantic") && in.attr.at("semantic") == "VERTEX") {
                        voff = off;
                        const std::string sid = strip_hash(in.attr.at("source"));
                        vsrc = vmap.count(sid) ? vmap[sid] : sid;
                    }
                }
                SubMesh sm;
                sm.name = prim.attr.count("material") ? prim.attr.at("material") : "";
                if (voff < 0 || !sources.count(vsrc)) {
                    m.submeshes.push_back(std::move(sm));
                    continue;
                }
                const auto &pos = sources[vsrc];
                const XNode *pn = prim.child("p");
                const std::vector<long> idx = pn ? parse_ints(pn->text) : std::vector<long>();
                std::vector<long> vc;
                if (prim.tag == "polylist") {
                    const XNode *vn = prim.child("vcount");
                    vc = vn ? parse_ints(vn->text) : std::vector<long>();
                } else {
                    vc.assign(idx.size() / stride / 3, 3);
                }
                size_t corner = 0;
                for (long c : vc) {
                    if (c == 3) {
                        for (int k = 0; k < 3; ++k) {
                            const size_t at = (corner + k) * stride + voff;
                            const long v = at < idx.size() ? idx[at] : -1;
                            if (v < 0 || (size_t)(3 * v + 2) >= pos.size()) {
                                m.error = true;
                                m.message = "dae: index out of range";
                                return m;
                            }
                            sm.tris.insert(sm.tris.end(), pos.begin() + 3 * v, pos.begin() + 3 * v + 3);
                        }
                    }
                    corner += (size_t)c;
                }
                m.submeshes.push_back(std::move(sm));
            }
        }
    return m;
}

// ------------------------------------------------------------------ 3DS (chunked binary)
struct Obj3ds {
    std::vector<float> verts;
    std::vector<uint16_t> faces;  // [n][3]
    std::vector<std::pair<std::string, std::vector<uint16_t>>> mats;
};

uint16_t rd16(const std::string &d, size_t o) { return (uint16_t)((uint8_t)d[o] | ((uint8_t)d[o + 1] << 8)); }
uint32_t rd32(const std::string &d, size_t o) {
    return (uint32_t)(uint8_t)d[o] | ((uint32_t)(uint8_t)d[o + 1] << 8) | ((uint32_t)(uint8_t)d[o + 2] << 16) |
           ((uint32_t)(uint8_t)d[o + 3] << 24);
}
std::string rdstr(const std::string &d, size_t o, size_t end, size_t &next) {
    size_t e = o;
    while (e < end && d[e] != 0) ++e;
    next = e + 1;
    return d.substr(o, e - o);
}

void walk3ds(const std::string &d, size_t off, size_t end, std::vector<std::string> &mats,
             std::vector<Obj3ds> &objs, Obj3ds *cur) {
    while (off + 6 <= end) {
        const uint16_t id = rd16(d, off);
        const uint32_t len = rd32(d, off + 2);
        if (len < 6 || off + len > end) return;
        const size_t body = off + 6, cend = off + len;
        size_t nx = 0;
        switch (id) {
            case 0x4D4D: case 0x3D3D: case 0x4100: case 0xAFFF:
                walk3ds(d, body, cend, mats, objs, cur);
                break;
            case 0xA000:
                mats.push_back(rdstr(d, body, cend, nx));
                break;
            case 0x4000: {
                objs.emplace_back();
                (void)rdstr(d, body, cend, nx);
                walk3ds(d, nx, cend, mats, objs, &objs.back());
                break;
            }
            // counts are clamped to what the chunk holds (a damaged file reads no further than
            // its chunk; sanitize_host.cpp feeds truncated and flipped files)
            case 0x4110:
                if (cur && body + 2 <= cend) {
                    const size_t n = std::min<size_t>(rd16(d, body), (cend - body - 2) / 12);
                    cur->verts.resize(3 * n);
                    if (n) std::memcpy(cur->verts.data(), d.data() + body + 2, sizeof(float) * 3 * n);
                }
                break;
            case 0x4120:
                if (cur && body + 2 <= cend) {
                    const size_t n = std::min<size_t>(rd16(d, body), (cend - body - 2) / 8);
                    cur->faces.resize(3 * n);
                    for (size_t f = 0; f < n; ++f)
                        for (int k = 0; k < 3; ++k) cur->faces[3 * f + k] = rd16(d, body + 2 + 8 * f + 2 * k);
                    walk3ds(d, body + 2 + 8 * n, cend, mats, objs, cur);
                }
                break;
            case 0x4130:
                if (cur) {
                    std::string name = rdstr(d, body, cend, nx);
                    if (nx + 2 > cend) break;
                    const size_t n = std::min<size_t>(rd16(d, nx), (cend - nx - 2) / 2);
                    std::vector<uint16_t> fl(n);
                    for (size_t f = 0; f < n; ++f) fl[f] = rd16(d, nx + 2 + 2 * f);
                    cur->mats.emplace_back(name, std::move(fl));
                }
                break;
            default:
                break;
        }
        off = cend;
    }
}

MeshFile load_3ds(const std::string &d) {
    MeshFile m;
    std::vector<std::string> mats;
    std::vector<Obj3ds> objs;
    walk3ds(d, 0, d.size(), mats, objs, nullptr);
    for (const auto &o : objs) {
        const size_t nf = o.faces.size() / 3;
        if (o.verts.empty() || nf == 0) continue;
        std::vector<size_t> fmat(nf, mats.size());  // faces without material: default, last
        for (const auto &mf : o.mats) {
            const auto it = std::find(mats.begin(), mats.end(), mf.first);
            const size_t mi = it == mats.end() ? mats.size() : (size_t)(it - mats.begin());
            for (uint16_t f : mf.second)
                if (f < nf) fmat[f] = mi;
        }
        for (size_t mi = 0; mi <= mats.size(); ++mi) {
            SubMesh sm;
            sm.name = mi < mats.size() ? mats[mi] : "DefaultMaterial";
            for (size_t f = 0; f < nf; ++f) {
                if (fmat[f] != mi) continue;
                bool inside = true;  // a face naming a missing vertex (damaged file) is dropped whole
                for (int k = 0; k < 3; ++k) inside = inside && 3 * (size_t)o.faces[3 * f + k] + 2 < o.verts.size();
                if (!inside) continue;
                for (int k = 0; k < 3; ++k) {
                    const size_t v = o.faces[3 * f + k];
                    for (int c = 0; c < 3; ++c) sm.tris.push_back((double)o.verts[3 * v + c]);
                }
            }
            if (!sm.tris.empty()) m.submeshes.push_back(std::move(sm));
        }
    }
    return m;
}

}  // namespace

MeshFile load_mesh(const std::string &path) {
    std::string text;
    MeshFile m;
    if (!read_file(path, text)) {
        m.error = true;
        m.message = "cannot open mesh file: " + path;
        return m;
    }
    const std::string e = lower_ext(path);
    if (e == "obj") return load_obj(text);
    if (e == "dae") return load_dae(text);
    if (e == "3ds") return load_3ds(text);
    m.error = true;
    m.message = "unsupported mesh format: " + path;
    return m;
}

}  // namespace mpt_host
