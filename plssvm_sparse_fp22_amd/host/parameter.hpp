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
#include <type_traits>
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

// plssvm::invalid_file_format_exception / file_not_found_exception (include/plssvm/exceptions/exceptions.hpp)
struct invalid_file_format_exception : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct file_not_found_exception : std::runtime_error {
    using std::runtime_error::runtime_error;
};

template <typename T>
constexpr const char *arithmetic_type_name() {  // include/plssvm/detail/arithmetic_type_name.hpp
    if constexpr (std::is_same_v<T, float>) return "float";
    else if constexpr (std::is_same_v<T, double>) return "double";
    else if constexpr (std::is_same_v<T, int>) return "int";
    else if constexpr (std::is_same_v<T, unsigned int>) return "unsigned int";
    else if constexpr (std::is_same_v<T, unsigned long>) return "unsigned long";
    else return "unsigned long long";
}

// detail::convert_to (include/plssvm/detail/string_conversion.hpp:39-64): leading whitespace skipped, the
// longest valid prefix converted (std::from_chars; correctly rounded like fast_float), error message verbatim
template <typename T>
T convert_to(std::string_view sv) {
    while (!sv.empty() && std::isspace((unsigned char) sv.front())) sv.remove_prefix(1);
    T v{};
    const auto r = std::from_chars(sv.data(), sv.data() + sv.size(), v);
    if (r.ec != std::errc{})
        throw invalid_file_format_exception("Can't convert '" + std::string(sv) + "' to a value of type " +
                                            arithmetic_type_name<T>() + "!");
    return v;
}

// a whole token as a real (data values: trailing characters are an error)
template <typename T>
T to_real(std::string_view sv) {
    while (!sv.empty() && std::isspace((unsigned char) sv.front())) sv.remove_prefix(1);
    while (!sv.empty() && std::isspace((unsigned char) sv.back())) sv.remove_suffix(1);
    T v{};
    const auto r = std::from_chars(sv.data(), sv.data() + sv.size(), v);  // correctly rounded, like fast_float
    if (r.ec != std::errc{} || r.ptr != sv.data() + sv.size())
        throw invalid_file_format_exception("Can't convert '" + std::string(sv) + "' to a value of type " +
                                            arithmetic_type_name<T>() + "!");
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
                    throw invalid_file_format_exception("Can't convert '" + std::string(idx) +
                                                        "' to a value of type unsigned long!");
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
        if (!f) throw file_not_found_exception("Couldn't find file: '" + filename + "'!");
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

    // parse_model_file (src/plssvm/parameter.cpp:366-520): the header lines (left-trimmed, '#' comments
    // skipped, lower-cased) until "sv", with the reference's checks and messages; then total_sv lines
    // "alpha idx:val ..." — the support vectors become this object's data, their alphas `alpha`, -rho the bias
    real_type rho = 0;
    std::vector<real_type> alpha;
    std::vector<int64_t> nr_sv;
    real_type label_first = 0, label_second = 0;
    void parse_model_file(const std::string &filename, bool keep_sparse = false, int64_t min_features = 0) {
        const std::string content = read_file(filename);
        // lines as detail::file_reader keeps them (file_reader.cpp:129-153)
        std::vector<std::string_view> lines;
        for (std::size_t pos = 0; pos <= content.size();) {
            std::size_t nl = content.find('\n', pos);
            if (nl == std::string::npos) nl = content.size();
            std::string_view l(content.data() + pos, nl - pos);
            pos = nl + 1;
            while (!l.empty() && std::isspace((unsigned char) l.front())) l.remove_prefix(1);
            if (!l.empty() && l.front() != '#') lines.push_back(l);
        }
        unsigned long long num_sv = 0;
        bool rho_set = false, nr_sv_set = false;
        label_first = label_second = 0;
        auto trim_left = [](std::string_view v) {
            while (!v.empty() && std::isspace((unsigned char) v.front())) v.remove_prefix(1);
            return v;
        };
        std::size_t header = 0;
        for (; header < lines.size(); ++header) {
            std::string_view raw = lines[header];
            while (!raw.empty() && std::isspace((unsigned char) raw.back())) raw.remove_suffix(1);
            std::string line(raw);
            std::transform(line.begin(), line.end(), line.begin(), [](unsigned char c) { return (char) std::tolower(c); });
            std::string_view value{ line };
            value.remove_prefix(std::min(value.find_first_of(' ') + 1, value.size()));
            value = trim_left(value);
            auto starts = [&](const char *k) { return line.rfind(k, 0) == 0; };
            if (starts("svm_type")) {
                if (value != "c_svc")
                    throw invalid_file_format_exception("Can only use c_svc as svm_type, but '" + std::string(value) +
                                                        "' was given!");
            } else if (starts("kernel_type")) {
                std::string_view tok = value.substr(0, value.find_first_of(' '));
                if (tok == "linear" || tok == "0") kernel = kernel_type::linear;
                else if (tok == "polynomial" || tok == "1") kernel = kernel_type::polynomial;
                else if (tok == "rbf" || tok == "2") kernel = kernel_type::rbf;
                else throw invalid_file_format_exception("Unrecognized kernel type '" + std::string(value) + "'!");
            } else if (starts("gamma")) {
                gamma = convert_to<real_type>(value);
            } else if (starts("degree")) {
                degree = convert_to<int>(value);
            } else if (starts("coef0")) {
                coef0 = convert_to<real_type>(value);
            } else if (starts("nr_class")) {
                const auto nr_class = convert_to<unsigned int>(value);
                if (nr_class != 2)
                    throw invalid_file_format_exception("Can only use 2 classes, but " + std::to_string(nr_class) +
                                                        " were given!");
            } else if (starts("total_sv")) {
                num_sv = convert_to<unsigned long long>(value);
                if (num_sv == 0)
                    throw invalid_file_format_exception("The number of support vectors must be greater than 0, but is 0!");
            } else if (starts("rho")) {
                rho = convert_to<real_type>(value);
                rho_set = true;
            } else if (starts("label")) {
                const std::string_view first = value.substr(0, value.find_first_of(' '));
                label_first = convert_to<real_type>(first);
                value.remove_prefix(std::min(first.size() + 1, value.size()));
                const std::string_view second = value.substr(0, value.find_first_of(" \n"));
                label_second = convert_to<real_type>(second);
                value.remove_prefix(std::min(second.size() + 1, value.size()));
                value = trim_left(value);
                if (!value.empty() || (label_first != 1 && label_first != -1) || (label_second != 1 && label_second != -1))
                    throw invalid_file_format_exception("Only the labels 1 and -1 are allowed, but '" + line +
                                                        "' were given!");
            } else if (starts("nr_sv")) {
                const std::string_view first = value.substr(0, value.find_first_of(' '));
                const auto a = convert_to<unsigned long long>(first);
                value.remove_prefix(std::min(first.size() + 1, value.size()));
                const std::string_view second = value.substr(0, value.find_first_of(" \n"));
                const auto b = convert_to<unsigned long long>(second);
                value.remove_prefix(std::min(second.size() + 1, value.size()));
                value = trim_left(value);
                if (!value.empty())
                    throw invalid_file_format_exception("Only two numbers are allowed, but more were given '" + line + "'!");
                if (a + b != num_sv)
                    throw invalid_file_format_exception(
                        "The number of positive and negative support vectors doesn't add up to the total number: " +
                        std::to_string(a) + " + " + std::to_string(b) + " != " + std::to_string(num_sv) + "!");
                nr_sv = { (int64_t) a, (int64_t) b };
                nr_sv_set = true;
            } else if (line == "sv") {
                break;
            } else {
                throw invalid_file_format_exception("Unrecognized header entry '" + std::string(raw) +
                                                    "'! Maybe SV is missing?");
            }
        }
        if (num_sv == 0) throw invalid_file_format_exception("Missing total number of support vectors!");
        if (label_first == 0 || label_second == 0) throw invalid_file_format_exception("Missing labels!");
        if (!nr_sv_set) throw invalid_file_format_exception("Missing number of support vectors per class!");
        if (!rho_set) throw invalid_file_format_exception("Missing rho value!");
        if (header + 1 >= lines.size())
            throw invalid_file_format_exception("Can't parse file: no support vectors are given or SV is missing!");
        if (lines.size() - header - 1 < num_sv)
            throw invalid_file_format_exception("total_sv is " + std::to_string(num_sv) + ", but only " +
                                                std::to_string(lines.size() - header - 1) +
                                                " support vectors are given!");
        // the support vector lines: exactly total_sv of them (parse_libsvm_content(f, header + 1, data(num_sv), ...))
        const std::size_t sv_begin = (std::size_t) (lines[header + 1].data() - content.data());
        const std::size_t sv_end = header + 1 + num_sv < lines.size()
                                       ? (std::size_t) (lines[header + 1 + num_sv].data() - content.data())
                                       : content.size();
        const rows_t pr = parse_rows(content.substr(0, sv_end), sv_begin);
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
