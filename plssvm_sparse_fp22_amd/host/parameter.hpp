// plssvm::mi355x::parameter<T> — training parameters + LIBSVM reader (C++17, host only).
//
// Mirrors plssvm::parameter<T> (include/plssvm/parameter.hpp:181-194 defaults; src/plssvm/parameter.cpp):
//   * LIBSVM lines left-trimmed, empty and '#' lines skipped (src/plssvm/detail/file_reader.cpp:129-153);
//   * label = token before the first space if it has no ':' (parameter.cpp:56-63), mapped by
//     sign (x > 0 ? +1 : -1, parameter.cpp:160-163);
//   * indices 0-based as written (parameter.cpp:75-83); num_features = max index + 1;
//   * gamma = 1 / num_features in the real type when not given (parameter.cpp:150-152);
//   * model file name = basename(input) + ".model", prediction file basename(input) + ".predict"
//     (parameter.cpp:575-584);
//   * model files as written by csvm::write_model (parameter.cpp:366-520).
// Unlike the reference, which always densifies, the data can be kept as CSR (`sparse = true`).
#pragma once

#include <algorithm>
#include <cctype>
#include <charconv>
#include <cstdint>
#include <cstdlib>
#include <cstring>
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
    std::vector<uint32_t> val22;    // packed FP22 words of `val` (binary FP22 input; kept packed for the device)
    std::vector<real_type> labels;  // +-1

    std::string predict_name_from_input() const {
        const auto pos = input_filename.find_last_of("/\\");
        return input_filename.substr(pos == std::string::npos ? 0 : pos + 1) + ".predict";
    }
    std::string model_name_from_input() const {
        const auto pos = input_filename.find_last_of("/\\");
        return input_filename.substr(pos == std::string::npos ? 0 : pos + 1) + ".model";
    }

    // LIBSVM rows "[label] idx:val ..." of content[start..] (parameter.cpp:40-176): left-trimmed, empty
    // and '#' lines skipped, a leading token without ':' is the label / alpha, indices 0-based
    struct rows_t {
        std::vector<std::vector<std::pair<int64_t, real_type>>> rows;
        std::vector<real_type> first;  // label (train / test) or alpha (model SV section)
        bool has_first = true;
    };
    static rows_t parse_rows(const std::string &content, std::size_t pos) {
        rows_t out;
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
                out.first.push_back(to_real<real_type>(line.substr(0, sp)));
                p = sp;
            } else {
                out.has_first = false;
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
            out.rows.push_back(std::move(r));
        }
        return out;
    }

    static std::string read_file(const std::string &filename) {
        std::ifstream f(filename, std::ios::binary);
        if (!f) throw std::runtime_error("Couldn't find file: '" + filename + "'!");
        std::stringstream ss;
        ss << f.rdbuf();
        return ss.str();
    }

    // the data of this parameter object from parsed rows (dense or CSR), d = max(min_features, max index + 1)
    void set_rows(const rows_t &pr, bool keep_sparse, int64_t min_features = 0) {
        const auto &rows = pr.rows;
        if (rows.empty()) throw invalid_file_format_exception("Can't parse file: no data points are given!");
        int64_t d = min_features;
        for (const auto &r : rows)
            if (!r.empty()) d = std::max<int64_t>(d, r.back().first + 1);
        if (d == 0) throw invalid_file_format_exception("Can't parse file: no data points are given!");
        num_data_points = (int64_t) rows.size();
        num_features = d;
        sparse = keep_sparse;
        rowptr.assign(1, 0);
        col.clear();
        val.clear();
        val22.clear();
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
                for (const auto &[c, v] : rows[(std::size_t) i]) dense[(std::size_t) (i * d + c)] = v;
        }
    }

    // PLSSVMB1 binary CSR / FP22 data file (layout: plssvm_sparse_fp22_amd/io.py); always kept sparse
    static bool is_binary(const std::string &content) { return content.size() >= 48 && content.compare(0, 8, "PLSSVMB1") == 0; }
    void parse_binary(const std::string &c) {
        auto rd = [&](std::size_t off, void *dst, std::size_t nb) {
            if (off + nb > c.size()) throw invalid_file_format_exception("truncated PLSSVMB1 file");
            std::memcpy(dst, c.data() + off, nb);
        };
        uint32_t vf[2];
        int64_t hdr[3];
        int32_t fmt[2];
        rd(8, vf, 8);
        rd(16, hdr, 24);
        rd(40, fmt, 8);
        if (vf[0] != 1) throw invalid_file_format_exception("unsupported PLSSVMB1 version");
        const int64_t n = hdr[0], d = hdr[1], nnz = hdr[2];
        if (n < 1 || d < 1 || nnz < 0) throw invalid_file_format_exception("Can't parse file: no data points are given!");
        auto pad8 = [](std::size_t b) { return (8 - b % 8) % 8; };
        std::size_t off = 48;
        rowptr.resize((std::size_t) n + 1);
        rd(off, rowptr.data(), 8 * ((std::size_t) n + 1));
        off += 8 * ((std::size_t) n + 1);
        col.resize((std::size_t) nnz);
        rd(off, col.data(), 4 * (std::size_t) nnz);
        off += 4 * (std::size_t) nnz + pad8(4 * (std::size_t) nnz);
        val.resize((std::size_t) nnz);
        val22.clear();
        std::size_t nb;
        if (fmt[0] == 2) {
            nb = 4 * 11 * (((std::size_t) nnz + 15) / 16);
            val22.resize(nb / 4 + 1, 0u);
            rd(off, val22.data(), nb);
            for (int64_t k = 0; k < nnz; ++k) {
                const int bit = 22 * (int) (k & 15);
                const uint32_t *w = val22.data() + (k >> 4) * 11 + (bit >> 5);
                const int sh = bit & 31;
                uint64_t x = (uint64_t) w[0] >> sh;
                if (sh > 10) x |= (uint64_t) w[1] << (32 - sh);
                const uint32_t u = (uint32_t) (x & 0x3FFFFFu) << 10;
                float f;
                std::memcpy(&f, &u, 4);
                val[(std::size_t) k] = (real_type) f;
            }
        } else if (fmt[0] == 1) {
            nb = 8 * (std::size_t) nnz;
            std::vector<double> tmp((std::size_t) nnz);
            rd(off, tmp.data(), nb);
            for (int64_t k = 0; k < nnz; ++k) val[(std::size_t) k] = (real_type) tmp[(std::size_t) k];
        } else {
            nb = 4 * (std::size_t) nnz;
            std::vector<float> tmp((std::size_t) nnz);
            rd(off, tmp.data(), nb);
            for (int64_t k = 0; k < nnz; ++k) val[(std::size_t) k] = (real_type) tmp[(std::size_t) k];
        }
        off += nb + pad8(nb);
        labels.clear();
        if (vf[1] & 1u) {
            std::vector<double> y((std::size_t) n);
            rd(off, y.data(), 8 * (std::size_t) n);
            for (const double v : y) labels.push_back(v > 0 ? real_type{ 1 } : real_type{ -1 });
        }
        if (rowptr[0] != 0 || rowptr.back() != nnz) throw invalid_file_format_exception("corrupt PLSSVMB1 row pointers");
        sparse = true;
        num_data_points = n;
        num_features = d;
        dense.clear();
    }

    // parse_train_file -> parse_libsvm_file (src/plssvm/parameter.cpp:132-176); PLSSVMB1 binary files too
    void parse_train_file(const std::string &filename, bool keep_sparse = false) {
        if (model_filename.empty() || model_filename == model_name_from_input()) {
            input_filename = filename;
            model_filename = model_name_from_input();
        }
        input_filename = filename;
        const std::string content = read_file(filename);
        if (is_binary(content)) {
            parse_binary(content);
            if (gamma == real_type{ 0 }) gamma = real_type{ 1 } / static_cast<real_type>(num_features);
            return;
        }
        const rows_t pr = parse_rows(content, 0);
        set_rows(pr, keep_sparse);
        if (gamma == real_type{ 0 }) gamma = real_type{ 1 } / static_cast<real_type>(num_features);
        labels.clear();
        if (pr.has_first && (int64_t) pr.first.size() == num_data_points)
            for (const real_type v : pr.first) labels.push_back(v > real_type{ 0 } ? real_type{ 1 } : real_type{ -1 });
    }

    // parse_test_file (parameter.cpp:132-176 on the test set): points + optional labels
    void parse_test_file(const std::string &filename, bool keep_sparse = false, int64_t min_features = 0) {
        const rows_t pr = parse_rows(read_file(filename), 0);
        set_rows(pr, keep_sparse, min_features);
        labels.clear();
        if (pr.has_first && (int64_t) pr.first.size() == num_data_points)
            for (const real_type v : pr.first) labels.push_back(v > real_type{ 0 } ? real_type{ 1 } : real_type{ -1 });
    }

    // parse_model_file (src/plssvm/parameter.cpp:366-520): header (kernel_type, degree, gamma, coef0,
    // rho, ...) until "SV", then one "alpha idx:val ..." line per support vector; the support vectors
    // become this object's data, their alphas `alpha`, -rho the bias
    real_type rho = 0;
    std::vector<real_type> alpha;
    void parse_model_file(const std::string &filename, bool keep_sparse = false, int64_t min_features = 0) {
        const std::string content = read_file(filename);
        std::size_t pos = 0;
        bool have_kernel = false, have_rho = false;
        while (true) {
            if (pos >= content.size()) throw invalid_file_format_exception("Can't parse file: no support vectors are given!");
            std::size_t nl = content.find('\n', pos);
            if (nl == std::string::npos) nl = content.size();
            std::string line(content.data() + pos, nl - pos);
            pos = nl + 1;
            while (!line.empty() && std::isspace((unsigned char) line.back())) line.pop_back();
            std::size_t b = 0;
            while (b < line.size() && std::isspace((unsigned char) line[b])) ++b;
            line = line.substr(b);
            if (line.empty()) continue;
            if (line == "SV") break;
            const std::size_t sp = line.find(' ');
            const std::string key = line.substr(0, sp), value = sp == std::string::npos ? "" : line.substr(sp + 1);
            if (key == "svm_type") {
                if (value != "c_svc") throw invalid_file_format_exception("Can only use c_svc as svm_type, but '" + value + "' was given!");
            } else if (key == "kernel_type") {
                kernel = parse_kernel(value);
                have_kernel = true;
            } else if (key == "degree") {
                degree = std::stoi(value);
            } else if (key == "gamma") {
                gamma = to_real<real_type>(value);
            } else if (key == "coef0") {
                coef0 = to_real<real_type>(value);
            } else if (key == "rho") {
                rho = to_real<real_type>(value);
                have_rho = true;
            } else if (key == "nr_class") {
                if (std::stoi(value) != 2) throw invalid_file_format_exception("Can only use 2 classes, but " + value + " were given!");
            } else if (key == "total_sv" || key == "label" || key == "nr_sv") {
                // informational (the SV section defines the support vectors)
            } else {
                throw invalid_file_format_exception("Unrecognized header entry '" + key + "'! Maybe SV is missing?");
            }
        }
        if (!have_kernel) throw invalid_file_format_exception("Missing kernel_type!");
        if (!have_rho) throw invalid_file_format_exception("Missing rho value!");
        const rows_t pr = parse_rows(content, pos);
        if (!pr.has_first || pr.first.size() != pr.rows.size())
            throw invalid_file_format_exception("Every support vector needs an alpha value!");
        set_rows(pr, keep_sparse, min_features);
        alpha = pr.first;
        if (gamma == real_type{ 0 }) gamma = real_type{ 1 } / static_cast<real_type>(num_features);
    }

    real_type value(int64_t i, int64_t f) const {  // feature f of point i (dense or CSR)
        if (!sparse) return dense[(std::size_t) (i * num_features + f)];
        const auto b = col.begin() + rowptr[i], e = col.begin() + rowptr[i + 1];
        const auto it = std::lower_bound(b, e, (int32_t) f);
        return (it != e && *it == f) ? val[(std::size_t) (it - col.begin())] : real_type{ 0 };
    }
};

}  // namespace plssvm::mi355x
