// Minimal cxxopts-style command line parsing shared by plssvm-train and plssvm-predict (the reference
// uses cxxopts v3.0.0: -x value, -xvalue, --long value, --long=value, positionals in order).
#pragma once

#include <map>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

struct cli {
    std::map<std::string, std::string> opt;
    std::vector<std::string> pos;
};

inline cli parse_cli(int argc, char **argv, const std::map<std::string, std::string> &shorts,
                     const std::set<std::string> &is_flag) {
    cli c;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        std::string key, val;
        bool has_val = false;
        if (a.rfind("--", 0) == 0) {
            key = a.substr(2);
            const auto eq = key.find('=');
            if (eq != std::string::npos) {
                val = key.substr(eq + 1);
                key = key.substr(0, eq);
                has_val = true;
            }
        } else if (a.size() >= 2 && a[0] == '-' && !(a[1] >= '0' && a[1] <= '9')) {
            const auto it = shorts.find(a.substr(1, 1));
            if (it == shorts.end()) throw std::invalid_argument("Option '" + a + "' does not exist");
            key = it->second;
            if (a.size() > 2) {
                val = a.substr(2);
                has_val = true;
            }
        } else {
            c.pos.push_back(a);
            continue;
        }
        if (is_flag.count(key)) {
            c.opt[key] = "1";
            continue;
        }
        if (!has_val) {
            if (i + 1 >= argc) throw std::invalid_argument("Option '" + key + "' is missing an argument");
            val = argv[++i];
        }
        c.opt[key] = val;
    }
    return c;
}

