// writeplotfile.cpp — plotfiles from decompressed boxes, without AMReX
// (src/writeplotfile.cpp:118-231, which calls amrex::WriteMultiLevelPlotfile
// on one rank).  The files are those AMReX writes for that call:
//
//   <out><name>/Header              plotfile header, reals at precision 17
//   <out><name>/Level_l/Cell_H      VisMF header: box array, FAB offsets,
//                                   per-FAB per-component min and max
//   <out><name>/Level_l/Cell_D_00000 every FAB of the level: one text header
//                                   line, then ncomp x W*H*D fp64, x fastest
//
// Geometry follows amrex::Geometry / RealBox arithmetic: level l's domain is
// (xDim, yDim, zDim) * ref_ratio^l cells, dx = (prob_hi - prob_lo) / n, and
// a box's physical extent is prob_lo + dx * lo .. prob_lo + dx * (hi + 1).
#include <array>
#include <cmath>
#include <cstdio>
#include <filesystem>
#include <fstream>
#include <sstream>

#include "log.h"
#include "wavelet_amd/writeplotfile.h"

using namespace wavelet_amd;

namespace {

std::string real17(double v) {
    char b[40];
    std::snprintf(b, sizeof b, "%.17g", v);
    return b;
}

std::string sci16(double v) {
    char b[40];
    std::snprintf(b, sizeof b, "%.16e", v);
    return b;
}

std::string box_str(const int lo[3], const int hi[3]) {
    std::ostringstream s;
    s << "((" << lo[0] << ',' << lo[1] << ',' << lo[2] << ") (" << hi[0] << ',' << hi[1] << ',' << hi[2]
      << ") (0,0,0))";
    return s.str();
}

constexpr const char* kFabReal = "FAB ((8, (64 11 52 0 1 12 0 1023)),(8, (8 7 6 5 4 3 2 1)))";

void write_level(const std::filesystem::path& ldir, const std::vector<Location>& locs,
                 const std::vector<Dimensions>& dims, std::vector<multiBox3D>& boxes, int ncomp) {
    std::filesystem::create_directories(ldir);
    const size_t nb = locs.size();
    if (boxes.size() < nb) {
        log_error("Index out of bounds: box_idx = " + std::to_string(boxes.size()) +
                  ", data.size() = " + std::to_string(boxes.size()));
        std::abort();
    }
    std::vector<uint64_t> offs(nb);
    std::vector<std::vector<double>> mins(nb, std::vector<double>(ncomp)), maxs(nb, std::vector<double>(ncomp));
    {
        std::ofstream d(ldir / "Cell_D_00000", std::ios::binary);
        std::vector<double> row;
        uint64_t pos = 0;
        for (size_t b = 0; b < nb; ++b) {
            const int lo[3] = {locs[b][0], locs[b][1], locs[b][2]};
            const int hi[3] = {lo[0] + dims[b][0] - 1, lo[1] + dims[b][1] - 1, lo[2] + dims[b][2] - 1};
            const std::string h = std::string(kFabReal) + box_str(lo, hi) + " " + std::to_string(ncomp) + "\n";
            offs[b] = pos;
            d.write(h.data(), (std::streamsize)h.size());
            pos += h.size();
            const size_t npts = (size_t)dims[b][0] * dims[b][1] * dims[b][2];
            row.resize(npts);
            for (int c = 0; c < ncomp; ++c) {
                const Box3D& src = boxes[b][c];
                // populateMF copies curr_box.get(i, j, k) cell by cell (src/writeplotfile.cpp:103-113)
                const float* s = src.data();
                double mn = INFINITY, mx = -INFINITY;
                for (size_t k = 0; k < npts; ++k) {
                    const double v = (double)s[k];
                    row[k] = v;
                    mn = v < mn ? v : mn;
                    mx = v > mx ? v : mx;
                }
                mins[b][c] = mn;
                maxs[b][c] = mx;
                d.write(reinterpret_cast<const char*>(row.data()), (std::streamsize)(8 * npts));
                pos += 8 * npts;
            }
        }
    }
    std::ofstream h(ldir / "Cell_H");
    h << "1\n1\n" << ncomp << "\n0\n";
    h << '(' << nb << " 0\n";
    for (size_t b = 0; b < nb; ++b) {
        const int lo[3] = {locs[b][0], locs[b][1], locs[b][2]};
        const int hi[3] = {lo[0] + dims[b][0] - 1, lo[1] + dims[b][1] - 1, lo[2] + dims[b][2] - 1};
        h << box_str(lo, hi) << '\n';
    }
    h << ")\n" << nb << '\n';
    for (size_t b = 0; b < nb; ++b) h << "FabOnDisk: Cell_D_00000 " << offs[b] << '\n';
    for (const auto* mm : {&mins, &maxs}) {
        h << '\n' << nb << ',' << ncomp << '\n';
        for (size_t b = 0; b < nb; ++b) {
            for (int c = 0; c < ncomp; ++c) h << sci16((*mm)[b][c]) << ',';
            h << '\n';
        }
    }
    h << '\n';
}

}  // namespace

void write_plotfiles(std::vector<std::vector<std::vector<multiBox3D>>> data, LocDimData locations,
                     LocDimData dimensions, std::vector<std::string> files, int num_levels, int num_components,
                     std::vector<std::string> comp_names, AMReXInfo amrexinfo, std::string out) {
    log_info("Writing the following plotfiles:");
    for (size_t t = 0; t < files.size(); ++t) {
        const std::string name = out + std::filesystem::path(files[t]).filename().string();
        log_info(name);
        if (!out.empty() && !std::filesystem::exists(out)) {
            std::error_code ec;
            std::filesystem::create_directories(out, ec);
            if (ec) log_error("Failed to create output directory " + out + ": " + ec.message());
        }
        const std::filesystem::path pdir(name);
        std::filesystem::create_directories(pdir);
        const double time = (double)amrexinfo.true_times[t];
        const std::vector<double>& g = amrexinfo.geomcellinfo[t];
        std::ostringstream H;
        H << "HyperCLaw-V1.1\n" << comp_names.size() << '\n';
        for (const auto& n : comp_names) H << n << '\n';
        H << 3 << '\n' << real17(time) << '\n' << num_levels - 1 << '\n';
        for (int k = 0; k < 3; ++k) H << real17(g[k]) << ' ';
        H << '\n';
        for (int k = 0; k < 3; ++k) H << real17(g[3 + k]) << ' ';
        H << '\n';
        for (int l = 1; l < num_levels; ++l) H << amrexinfo.ref_ratios[0] << ' ';
        H << '\n';
        std::vector<std::array<int, 3>> ncell(num_levels);
        std::vector<std::array<double, 3>> dx(num_levels);
        const int base[3] = {amrexinfo.xDim, amrexinfo.yDim, amrexinfo.zDim};
        for (int l = 0; l < num_levels; ++l)
            for (int k = 0; k < 3; ++k) {
                ncell[l][k] = (int)(base[k] * std::pow(amrexinfo.ref_ratios[k], l));
                dx[l][k] = (g[3 + k] - g[k]) / (double)ncell[l][k];
            }
        for (int l = 0; l < num_levels; ++l) {
            const int lo[3] = {0, 0, 0};
            const int hi[3] = {ncell[l][0] - 1, ncell[l][1] - 1, ncell[l][2] - 1};
            H << box_str(lo, hi) << ' ';
        }
        H << '\n';
        for (int l = 0; l < num_levels; ++l) H << amrexinfo.level_steps[t][l] << ' ';
        H << '\n';
        for (int l = 0; l < num_levels; ++l) {
            for (int k = 0; k < 3; ++k) H << real17(dx[l][k]) << ' ';
            H << '\n';
        }
        H << "0\n0\n";  // Cartesian coordinates; boundary width
        for (int l = 0; l < num_levels; ++l) {
            const auto& locs = locations[t][l];
            const auto& dims = dimensions[t][l];
            H << l << ' ' << locs.size() << ' ' << real17(time) << '\n' << amrexinfo.level_steps[t][l] << '\n';
            for (size_t b = 0; b < locs.size(); ++b)
                for (int k = 0; k < 3; ++k) {
                    const double lo = g[k] + dx[l][k] * locs[b][k];
                    const double hi = g[k] + dx[l][k] * (locs[b][k] + dims[b][k]);
                    H << real17(lo) << ' ' << real17(hi) << '\n';
                }
            H << "Level_" << l << "/Cell\n";
            write_level(pdir / ("Level_" + std::to_string(l)), locs, dims, data[t][l], num_components);
        }
        std::ofstream hf(pdir / "Header");
        const std::string hs = H.str();
        hf.write(hs.data(), (std::streamsize)hs.size());
    }
}
