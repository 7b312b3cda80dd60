// plssvm::mi355x::parameter<T> — training parameters + LIBSVM reader (C++17, host only).
//
// Mirrors plssvm::parameter<T> (include/plssvm/parameter.hpp:181-194 defaults; src/plssvm/parameter.cpp):
//   * LIBSVM lines left-trimmed, empty and '#' lines skipped (src/plssvm/detail/file_reader.cpp:129-153);
//   * label = token before the first space if it has no ':' (parameter.cpp:56-63), mapped by
//     sign (x > 0 ? +1 : -1, parameter.cpp:160-163);
//   * indices 0-based as written (parameter.cpp:75-83); num_features = max index + 1;
//   * gamma = 1 / num_features in the real type when not given (parameter.cpp:150-152);
//   * model file name = basename(input) + ".model" (parameter.cpp:575-578).
// Unlike the reference, which always densifies, the data can be kept as CSR (`sparse = true`).
#pragma once

#include <algorithm>
#include <cctype>
#include <charconv>
#include <cstdint>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace plssvm::mi355x {

enum class kernel_type { linear = 0, polynomial = 1, rbf = 2 };

inline const char *kernel_name(kernel_type k) {
    switch (k) {
        case kernel_type::linear: return "linear";
        case kernel_type::polynomial: return "polynomial";
        default: return "rbf";
    }
}

inline kernel_type parse_kernel(std::string s) {
    std::transform(s.begin(), s.end(), s.begin(), [](unsigned char c) { return (char) std::tolower(c); });
    if (s == "linear" || s == "0") return kernel_type::linear;
    if (s == "polynomial" || s == "1") return kernel_type::polynomial;
    if (s == "rbf" || s == "2") return kernel_type::rbf;
    throw std::invalid_argument("Unrecognized kernel type '" + s + "'!");
}

struct invalid_file_format_exception : std::runtime_error {
    using std::runtime_error::runtime_error;
};

template <typename T>
T to_real(std::string_view sv) {
    while (!sv.empty() && std::isspace((unsigned char) sv.front())) sv.remove_prefix(1);
    while (!sv.empty() && std::isspace((unsigned char) sv.back())) sv.remove_suffix(1);
    T v{};
    const auto r = std::from_chars(sv.data(), sv.data() + sv.size(), v);  // correctly rounded, like fast_float
    if (r.ec != std::errc{} || r.ptr != sv.data() + sv.size())
        throw invalid_file_format_exception("Can't convert '" + std::string(sv) + "' to a floating point value!");
    return v;
}

template <typename T>
struct parameter {
    using real_type = T;
    kernel_type kernel = kernel_type::linear;
    int degree = 3;
    real_type gamma = 0;  // 0 -> 1 / num_features
    real_type coef0 = 0;
    real_type cost = 1;
    real_type epsilon = 0.001;
    bool print_info = true;
    std::string input_filename, model_filename;

    // data: dense rows (row-major n x d) or CSR
    bool sparse = false;
    int64_t num_data_points = 0, num_features = 0;
    std::vector<real_type> dense;
    std::vector<int64_t> rowptr;
    std::vector<int32_t> col;
    std::vector<real_type> val;
    std::vector<real_type> labels;  // +-1

    std::string model_name_from_input() const {
        const auto pos = input_filename.find_last_of("/\\");
        return input_filename.substr(pos == std::string::npos ? 0 : pos + 1) + ".model";
    }

    // parse_train_file -> parse_libsvm_file (src/plssvm/parameter.cpp:132-176)
    void parse_train_file(const std::string &filename, bool keep_sparse = false) {
        if (model_filename.empty() || model_filename == model_name_from_input()) {
            input_filename = filename;
            model_filename = model_name_from_input();
        }
        input_filename = filename;
        std::ifstream f(filename, std::ios::binary);
        if (!f) throw std::runtime_error("Couldn't find file: '" + filename + "'!");
        std::stringstream ss;
        ss << f.rdbuf();
        const std::string content = ss.str();

        std::vector<std::vector<std::pair<int64_t, real_type>>> rows;
        std::vector<real_type> vals;
        bool has_label = true;
        std::size_t pos = 0;
        while (pos <= content.size()) {
            std::size_t nl = content.find('\n', pos);
            if (nl == std::string::npos) nl = content.size();
            std::string_view line(content.data() + pos, nl - pos);
            pos = nl + 1;
            while (!line.empty() && std::isspace((unsigned char) line.front())) line.remove_prefix(1);
            if (line.empty() || line.front() == '#') continue;
            std::size_t sp = line.find_first_of(" \n");
            const std::size_t colon = line.find_first_of(":\n");
            std::size_t p = 0;
            if (sp == std::string_view::npos) sp = line.size();
            if (colon == std::string_view::npos || colon >= sp) {
                vals.push_back(to_real<real_type>(line.substr(0, sp)));
                p = sp;
            } else {
                has_label = false;
            }
            std::vector<std::pair<int64_t, real_type>> r;
            while (true) {
                const std::size_t c = line.find(':', p);
                if (c == std::string_view::npos) break;
                std::string_view idx = line.substr(p, c - p);
                while (!idx.empty() && std::isspace((unsigned char) idx.front())) idx.remove_prefix(1);
                unsigned long index = 0;
                const auto res = std::from_chars(idx.data(), idx.data() + idx.size(), index);
                if (res.ec != std::errc{})
                    throw invalid_file_format_exception("Can't convert '" + std::string(idx) + "' to an index!");
                p = c + 1;
                std::size_t e = line.find(' ', p);
                if (e == std::string_view::npos) e = line.size();
                r.emplace_back((int64_t) index, to_real<real_type>(line.substr(p, e - p)));
                p = e;
            }
            std::sort(r.begin(), r.end());
            rows.push_back(std::move(r));
        }
        if (rows.empty()) throw invalid_file_format_exception("Can't parse file: no data points are given!");
        int64_t d = 0;
        for (const auto &r : rows)
            if (!r.empty()) d = std::max<int64_t>(d, r.back().first + 1);
        if (d == 0) throw invalid_file_format_exception("Can't parse file: no data points are given!");
        num_data_points = (int64_t) rows.size();
        num_features = d;
        if (gamma == real_type{ 0 }) gamma = real_type{ 1 } / static_cast<real_type>(d);
        labels.clear();
        if (has_label && (int64_t) vals.size() == num_data_points)
            for (const real_type v : vals) labels.push_back(v > real_type{ 0 } ? real_type{ 1 } : real_type{ -1 });
        sparse = keep_sparse;
        rowptr.assign(1, 0);
        col.clear();
        val.clear();
        dense.clear();
        if (sparse) {
            for (const auto &r : rows) {
                for (const auto &[c, v] : r) {
                    col.push_back((int32_t) c);
                    val.push_back(v);
                }
                rowptr.push_back((int64_t) col.size());
            }
        } else {
            dense.assign((std::size_t) (num_data_points * d), real_type{ 0 });
            for (int64_t i = 0; i < num_data_points; ++i)
                for (const auto &[c, v] : rows[i]) dense[(std::size_t) (i * d + c)] = v;
        }
    }

    real_type value(int64_t i, int64_t f) const {  // feature f of point i (dense or CSR)
        if (!sparse) return dense[(std::size_t) (i * num_features + f)];
        const auto b = col.begin() + rowptr[i], e = col.begin() + rowptr[i + 1];
        const auto it = std::lower_bound(b, e, (int32_t) f);
        return (it != e && *it == f) ? val[(std::size_t) (it - col.begin())] : real_type{ 0 };
    }
};

}  // namespace plssvm::mi355x
