// argparse.cpp — run parameters and input selection (src/argparse.cpp:10-178).
//
// Parameters: the reference queries amrex::ParmParse, which amrex::Initialize
// fills from the command line: the arguments are joined with spaces and read
// as `name = value value ...` definitions, a definition's values running up to
// the token before the next `=`; a query returns the last definition.  A
// missing parameter is logged and the run continues (src/argparse.cpp:17-68).
#include <algorithm>
#include <cctype>
#include <filesystem>
#include <limits>
#include <map>
#include <sstream>

#include "log.h"
#include "wavelet_amd/argparse.h"
#include "wavelet_amd/xz_pool.h"

using namespace wavelet_amd;

namespace {

std::map<std::string, std::vector<std::string>>& params() {
    static std::map<std::string, std::vector<std::string>> table;
    return table;
}

// split on whitespace, '=' as a token of its own
std::vector<std::string> tokenize(const std::string& s) {
    std::vector<std::string> out;
    std::string cur;
    auto flush = [&]() {
        if (!cur.empty()) out.push_back(cur);
        cur.clear();
    };
    for (char ch : s) {
        if (std::isspace(static_cast<unsigned char>(ch))) {
            flush();
        } else if (ch == '=') {
            flush();
            out.emplace_back("=");
        } else {
            cur.push_back(ch);
        }
    }
    flush();
    return out;
}

template <class T>
bool query(const std::string& name, T& v) {
    auto it = params().find(name);
    if (it == params().end() || it->second.empty()) return false;
    std::istringstream is(it->second.front());
    T tmp{};
    if (!(is >> tmp)) return false;
    v = tmp;
    return true;
}

bool query(const std::string& name, std::string& v) {
    auto it = params().find(name);
    if (it == params().end() || it->second.empty()) return false;
    v = it->second.front();
    return true;
}

bool queryarr(const std::string& name, std::vector<std::string>& v) {
    auto it = params().find(name);
    if (it == params().end()) return false;
    v = it->second;
    return true;
}

}  // namespace

void init_params(int argc, char* argv[]) {
    std::string joined;
    for (int i = 1; i < argc; ++i) {
        joined += argv[i];
        joined += ' ';
    }
    const std::vector<std::string> tok = tokenize(joined);
    params().clear();
    for (size_t i = 0; i + 1 < tok.size(); ++i) {
        if (tok[i] == "=" || tok[i + 1] != "=") continue;
        std::vector<std::string> vals;
        size_t j = i + 2;
        while (j < tok.size() && !(j + 1 < tok.size() && tok[j + 1] == "=") && tok[j] != "=") vals.push_back(tok[j++]);
        params()[tok[i]] = vals;  // a later definition replaces an earlier one
        i = j - 1;
    }
}

Config parse_config_compress() {
    Config cfg;
    if (!query("datadir", cfg.data_dir)) log_error("Missing datadir!");
    if (!query("minfile", cfg.min_time)) log_error("Missing minfile!");
    if (!query("maxfile", cfg.max_time)) log_error("Missing maxfile!");
    if (!query("minlevel", cfg.min_level)) log_error("Missing minlevel!");
    if (!query("maxlevel", cfg.max_level)) log_error("Missing maxlevel!");
    if (!queryarr("components", cfg.components)) log_error("Missing component list!");
    if (!query("keep", cfg.keep)) log_error("Missing 'keep' parameter!");
    if (!query("compresseddir", cfg.compressed_dir)) log_error("Missing compresseddir!");
    std::string preset;  // optional, not a reference parameter: no error when absent
    if (query("xzpreset", preset)) {
        cfg.xz_preset = parse_xz_preset(preset.c_str());
        if (cfg.xz_preset < 0) log_error("Bad xzpreset (0-9, optionally followed by e): " + preset);
    }
    return cfg;
}

Config parse_config_decompress() {
    Config cfg;
    if (!query("compresseddir", cfg.compressed_dir)) log_error("Missing compresseddir!");
    if (!query("out", cfg.out_dir)) log_error("Missing out directory!");
    return cfg;
}

bool has_flag(int argc, char* argv[], const std::string& flag) {
    for (int i = 1; i < argc; ++i)
        if (flag == argv[i]) return true;
    return false;
}

int clean_string(std::string filename) {
    std::string digits;
    for (char ch : filename)
        if (std::isdigit(static_cast<unsigned char>(ch))) digits.push_back(ch);
    if (digits.empty()) return -1;
    const size_t nz = digits.find_first_not_of('0');
    if (nz == std::string::npos) return 0;
    // The reference's std::stoi throws std::out_of_range (an uncaught
    // terminate) once the digits pass INT_MAX, which the digits of a whole
    // path easily do (a temp directory's random name): saturate instead, so
    // such a path simply matches no time range.
    const std::string d = digits.substr(nz);
    if (d.size() > 10 || (d.size() == 10 && d > "2147483647")) return std::numeric_limits<int>::max();
    return std::stoi(d);
}

std::vector<std::string> format_files(std::string data_dir, std::string min_time, std::string max_time) {
    const int first = clean_string(min_time), last = clean_string(max_time);
    std::vector<std::string> files;
    log_info("This run involves the following files:");
    for (const auto& e : std::filesystem::directory_iterator(data_dir)) {
        // the digits of the WHOLE path count, as in the reference
        const int cur = clean_string(e.path().string());
        if (cur >= first && cur <= last) files.push_back(e.path().string());
    }
    std::sort(files.begin(), files.end());  // deterministic order for equal keys
    std::stable_sort(files.begin(), files.end(),
                     [](const std::string& a, const std::string& b) { return clean_string(a) < clean_string(b); });
    for (const auto& f : files) log_info(f);
    return files;
}

std::vector<int> format_levels(int min_level, int max_level) {
    std::vector<int> levels;
    for (int l = min_level; l <= max_level; ++l) levels.push_back(l);
    return levels;
}
