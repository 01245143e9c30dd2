// readandwrite.cpp — the run's .raw side files (src/readandwrite.cpp:10-395).
// Same bytes as the reference: native little-endian; strings and vectors
// prefixed by a size_t count; locations, dimensions and box counts stored as
// float32; true times as x87 long double in 16 bytes; files named by plain
// string concatenation path + name (so `path` carries its trailing '/').
#include <cstdint>
#include <cstring>
#include <fstream>

#include "log.h"
#include "wavelet_amd/readandwrite.h"

using namespace wavelet_amd;

namespace {

class Out {
public:
    Out(const std::string& path, const std::string& name) : f_(path + name, std::ios::binary) {
        if (!f_.is_open()) {
            log_error("Failed to open file: " + path + name);
            std::exit(EXIT_FAILURE);
        }
    }
    template <class T>
    void pod(const T& v) {
        f_.write(reinterpret_cast<const char*>(&v), sizeof(T));
    }
    void f32(float v) { pod(v); }
    void i32(int v) { pod(v); }
    void count(size_t n) { pod(n); }
    void ld(long double v) {
        unsigned char b[sizeof(long double)] = {};  // padding bytes written as zero
        std::memcpy(b, &v, 10);                        // x87 80-bit value
        f_.write(reinterpret_cast<const char*>(b), sizeof b);
    }
    void str(const std::string& s) {
        count(s.size());
        f_.write(s.data(), (std::streamsize)s.size());
    }

private:
    std::ofstream f_;
};

class In {
public:
    In(const std::string& path, const std::string& name) : f_(path + name, std::ios::binary) {
        if (!f_.is_open()) {
            log_error("Failed to open file: " + path + name);
            std::exit(EXIT_FAILURE);
        }
    }
    template <class T>
    T pod() {
        T v{};
        f_.read(reinterpret_cast<char*>(&v), sizeof(T));
        return v;
    }
    float f32() { return pod<float>(); }
    int i32() { return pod<int>(); }
    size_t count() { return pod<size_t>(); }
    long double ld() { return pod<long double>(); }
    std::string str() {
        const size_t n = count();
        std::string s(n, '\0');
        f_.read(s.data(), (std::streamsize)n);
        return s;
    }

private:
    std::ifstream f_;
};

}  // namespace

void write_loc_dim_to_bin(LocDimData data, std::string path, std::string out_file, AMRIterator iterator) {
    Out o(path, out_file);
    iterator.iterate([&](int t, int lev, int b) {
        for (int k = 0; k < 3; ++k) o.f32((float)data[t][lev][b][k]);
    });
}

LocDimData read_loc_dim_from_bin(std::string const& path, std::string const& in_file,
                                 std::vector<std::vector<int>> /*counts*/, AMRIterator iterator, int num_times,
                                 int num_levels) {
    In in(path, in_file);
    LocDimData out(num_times, std::vector<std::vector<std::vector<int>>>(num_levels));
    iterator.iterate([&](int t, int lev, int) {
        std::vector<int> v(3);
        for (int k = 0; k < 3; ++k) v[k] = (int)in.f32();
        out[t][lev].push_back(std::move(v));
    });
    return out;
}

void write_box_counts(std::vector<std::vector<int>> counts, std::string const& path, std::string const& out_file,
                      int num_times, int num_levels) {
    Out o(path, out_file);
    for (int t = 0; t < num_times; ++t)
        for (int l = 0; l < num_levels; ++l) o.f32((float)counts.at(t).at(l));
}

std::vector<std::vector<int>> read_box_counts(std::string path, std::string in_file, int num_times,
                                              int num_levels) {
    In in(path, in_file);
    std::vector<std::vector<int>> out(num_times, std::vector<int>(num_levels));
    for (int t = 0; t < num_times; ++t)
        for (int l = 0; l < num_levels; ++l) out[t][l] = (int)in.f32();
    return out;
}

void write_amrexinfo(AMReXInfo info, std::string path, std::string out_file) {
    Out o(path, out_file);
    o.count(info.geomcellinfo.size());
    for (const auto& v : info.geomcellinfo) {
        o.count(v.size());
        for (double d : v) o.pod(d);
    }
    o.count(info.ref_ratios.size());
    for (int r : info.ref_ratios) o.i32(r);
    o.count(info.true_times.size());
    for (long double t : info.true_times) o.ld(t);
    o.count(info.level_steps.size());
    for (const auto& v : info.level_steps) {
        o.count(v.size());
        for (int s : v) o.i32(s);
    }
    o.i32(info.xDim);
    o.i32(info.yDim);
    o.i32(info.zDim);
}

AMReXInfo read_amrex_info(std::string path, std::string in_file) {
    In in(path, in_file);
    AMReXInfo info;
    info.geomcellinfo.resize(in.count());
    for (auto& v : info.geomcellinfo) {
        v.resize(in.count());
        for (double& d : v) d = in.pod<double>();
    }
    info.ref_ratios.resize(in.count());
    for (int& r : info.ref_ratios) r = in.i32();
    info.true_times.resize(in.count());
    for (long double& t : info.true_times) t = in.ld();
    info.level_steps.resize(in.count());
    for (auto& v : info.level_steps) {
        v.resize(in.count());
        for (int& s : v) s = in.i32();
    }
    info.xDim = in.i32();
    info.yDim = in.i32();
    info.zDim = in.i32();
    return info;
}

void write_runinfo(RunInfo info, std::string path, std::string out_file) {
    Out o(path, out_file);
    o.count(info.files.size());
    for (const auto& f : info.files) o.str(f);
    o.i32(info.min_level);
    o.i32(info.max_level);
    o.count(info.components.size());
    for (const auto& c : info.components) o.str(c);
    o.count(info.comp_idxs.size());
    for (int c : info.comp_idxs) o.i32(c);
}

RunInfo read_runinfo(std::string path, std::string in_file) {
    In in(path, in_file);
    RunInfo info;
    info.files.resize(in.count());
    for (auto& f : info.files) f = in.str();
    info.min_level = in.i32();
    info.max_level = in.i32();
    info.components.resize(in.count());
    for (auto& c : info.components) c = in.str();
    info.comp_idxs.resize(in.count());
    for (int& c : info.comp_idxs) c = in.i32();
    return info;
}
