// instance_file_map.hpp -- the `.inst` entry point (utilities/instancefilemap.hpp:11-84).
// Format: one `Key ? value` per line; key = text before the first '?', value = the rest,
// both trimmed; a line without '?' maps to itself (instancefilemap.hpp:23-35).
// Difference at the boundary: a missing key throws std::runtime_error instead of exit(1)
// (instancefilemap.hpp:45-47), so the C ABI never terminates the host process.
#pragma once
#include <cctype>
#include <fstream>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace mpt_host {

class InstanceFileMap {
public:
    explicit InstanceFileMap(const std::string &instance) : path_(instance) {
        std::ifstream file(instance.c_str());
        if (!file.is_open()) throw std::runtime_error("can't open instance file: " + instance);
        std::string line;
        while (std::getline(file, line)) {
            const auto delim = line.find('?');
            if (delim == std::string::npos) {
                map_[line] = line;
            } else {
                map_[trim(line.substr(0, delim))] = trim(line.substr(delim + 1));
            }
        }
    }

    bool exists(const std::string &key) const { return map_.find(key) != map_.end(); }

    const std::string &value(const std::string &key) const {
        const auto it = map_.find(key);
        if (it == map_.end()) throw std::runtime_error("Key \"" + key + "\" not bound");
        return it->second;
    }

    std::string value_or(const std::string &key, const std::string &dflt) const {
        return exists(key) ? value(key) : dflt;
    }

    std::vector<std::string> valueList(const std::string &key, const std::string &delim = " ") const {
        std::vector<std::string> out;
        const std::string &v = value(key);
        size_t i = 0;
        while (i < v.size()) {
            while (i < v.size() && delim.find(v[i]) != std::string::npos) ++i;
            size_t j = i;
            while (j < v.size() && delim.find(v[j]) == std::string::npos) ++j;
            if (j > i) out.push_back(v.substr(i, j - i));
            i = j;
        }
        return out;
    }

    std::vector<double> doubles(const std::string &key) const {
        std::vector<double> out;
        for (const auto &t : valueList(key)) out.push_back(std::stod(t));
        return out;
    }

    // Resolve a mesh path: absolute, else relative to the .inst directory, else as given.
    std::string resolve(const std::string &p) const {
        if (!p.empty() && p[0] == '/') return p;
        const auto slash = path_.find_last_of('/');
        const std::string dir = slash == std::string::npos ? std::string(".") : path_.substr(0, slash);
        const std::string cand = dir + "/" + p;
        std::ifstream f(cand.c_str());
        return f.good() ? cand : p;
    }

private:
    static std::string trim(std::string s) {
        size_t a = 0, b = s.size();
        while (a < b && std::isspace((unsigned char)s[a])) ++a;
        while (b > a && std::isspace((unsigned char)s[b - 1])) --b;
        return s.substr(a, b - a);
    }
    std::string path_;
    std::unordered_map<std::string, std::string> map_;
};

}  // namespace mpt_host
