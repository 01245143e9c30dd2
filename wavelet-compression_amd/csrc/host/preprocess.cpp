// preprocess.cpp — AMReX plotfile reading without AMReX.
//
//   read_plot_header  src/preprocess.cpp:131-242 (Header: names, dim, time,
//                     prob_lo/hi, ref ratios, level-0 domain, level steps)
//   read_level_index  amrex::VisMF::Read's view of Level_N/Cell_H (src/preprocess.cpp:36)
//   read_fab          one FAB of Cell_D_xxxxx: text header line, then
//                     ncomp x (x-fastest W*H*D) IEEE fp64 values
//   preprocess_data   src/preprocess.cpp:107-307, same outputs and quirks
//                     (max initialised to FLT_MIN, components in Header order,
//                     level steps = the first levels.size() values)
#include <algorithm>
#include <cfloat>
#include <cstring>
#include <fstream>
#include <sstream>

#include "log.h"
#include "wavelet_amd/preprocess.h"

namespace wavelet_amd {

PlotHeader read_plot_header(const std::string& plotfile) {
    PlotHeader h;
    std::ifstream x(plotfile + "/Header");
    if (!x.is_open()) {
        log_error("Failed to open header file: " + plotfile);
        std::exit(EXIT_FAILURE);
    }
    std::string str;
    int ncomp = 0;
    x >> str >> ncomp;
    for (int n = 0; n < ncomp; ++n) {
        x >> str;
        h.names.push_back(str);
    }
    x >> h.dim;
    std::getline(x, str);
    x >> h.true_time;
    std::getline(x, str);
    std::getline(x, str);  // finest level
    h.geomcell.assign(6, 0.0);
    for (int half = 0; half < 2; ++half) {
        std::getline(x, str);
        std::istringstream is(str);
        double a = 0, b = 0, c = 0;
        is >> a >> b >> c;
        h.geomcell[3 * half] = a;
        h.geomcell[3 * half + 1] = b;
        h.geomcell[3 * half + 2] = c;
    }
    std::getline(x, str);  // refinement ratios, one per coarser level (empty with one level)
    {
        // The reference extracts `dim` ints into one uninitialised local; once
        // the line runs out the extraction does nothing and the last value
        // stays, so "2 " reads as {2, 2, 2} (its Preprocessing test expects
        // exactly that).  A value missing from the start reads as 0 here.
        std::istringstream is(str);
        h.ref_ratios.assign(std::max(h.dim, 0), 0);
        int v = 0;
        for (int& r : h.ref_ratios) {
            is >> v;
            r = v;
        }
    }
    std::getline(x, str);  // level domains: ((lo) (hi) (type)) ...; the level-0 hi is after the third '('
    {
        size_t p = str.find('(');
        p = str.find('(', p + 1);
        p = str.find('(', p + 1);
        const size_t e = str.find(')', p);
        if (p == std::string::npos || e == std::string::npos) {
            log_error("Malformed domain line in " + plotfile + "/Header");
            std::exit(EXIT_FAILURE);
        }
        std::istringstream is(str.substr(p + 1, e - p));
        std::string v;
        std::vector<int> dims;
        while (std::getline(is, v, ',')) dims.push_back(std::stoi(v));
        if (dims.size() < 3) {
            log_error("Malformed domain line in " + plotfile + "/Header");
            std::exit(EXIT_FAILURE);
        }
        h.xDim = dims[0] + 1;
        h.yDim = dims[1] + 1;
        h.zDim = dims[2] + 1;
    }
    std::getline(x, str);
    {
        std::istringstream is(str);
        int v;
        while (is >> v) h.steps.push_back(v);
    }
    return h;
}

std::vector<int> match_components(const PlotHeader& h, const std::vector<std::string>& components) {
    std::vector<int> idx;
    for (int n = 0; n < (int)h.names.size(); ++n)
        if (std::find(components.begin(), components.end(), h.names[n]) != components.end()) idx.push_back(n);
    if (idx.size() != components.size()) return {};
    return idx;
}

// "FAB ((8, (64 11 52 0 1 12 0 1023)),(8, (8 7 6 5 4 3 2 1)))((lo) (hi) (t)) ncomp"
static bool parse_fab_header(const std::string& line, FabRef& f) {
    const size_t ord = line.find(",(");
    const size_t ordv = ord == std::string::npos ? ord : line.find('(', ord + 2);
    if (line.compare(0, 6, "FAB ((") != 0 || ordv == std::string::npos) return false;
    const int nbytes = std::atoi(line.c_str() + 6);
    int order[8];
    if (nbytes != 8 || std::sscanf(line.c_str() + ordv + 1, "%d %d %d %d %d %d %d %d", &order[0], &order[1],
                                   &order[2], &order[3], &order[4], &order[5], &order[6], &order[7]) != 8)
        return false;
    bool le = true, be = true;
    for (int i = 0; i < 8; ++i) {
        le = le && order[i] == 8 - i;
        be = be && order[i] == i + 1;
    }
    if (!le && !be) return false;
    f.big_endian = be;
    const size_t box = line.find(")))(");
    if (box == std::string::npos) return false;
    int t[3];
    if (std::sscanf(line.c_str() + box + 3, "((%d,%d,%d) (%d,%d,%d) (%d,%d,%d)) %d", &f.lo[0], &f.lo[1], &f.lo[2],
                    &f.hi[0], &f.hi[1], &f.hi[2], &t[0], &t[1], &t[2], &f.ncomp) != 10)
        return false;
    return true;
}

std::vector<FabRef> read_level_index(const std::string& plotfile, int level) {
    const std::string ldir = plotfile + "/Level_" + std::to_string(level) + "/";
    std::ifstream h(ldir + "Cell_H");
    if (!h.is_open()) {
        log_error("Failed to open " + ldir + "Cell_H");
        std::exit(EXIT_FAILURE);
    }
    std::vector<FabRef> out;
    std::string line;
    while (std::getline(h, line)) {
        if (line.compare(0, 10, "FabOnDisk:") != 0) continue;
        std::istringstream is(line.substr(10));
        FabRef f{};
        is >> f.file >> f.offset;
        f.file = ldir + f.file;
        std::ifstream d(f.file, std::ios::binary);
        std::string fh;
        if (!d.is_open() || !d.seekg((std::streamoff)f.offset) || !std::getline(d, fh) || !parse_fab_header(fh, f)) {
            log_error("Unreadable FAB in " + f.file);
            std::exit(EXIT_FAILURE);
        }
        out.push_back(f);
    }
    return out;
}

void read_fab(const FabRef& fab, const std::vector<int>& comps, double* dst) {
    std::ifstream d(fab.file, std::ios::binary);
    std::string fh;
    if (!d.is_open() || !d.seekg((std::streamoff)fab.offset) || !std::getline(d, fh)) {
        log_error("Failed to read FAB in " + fab.file);
        std::exit(EXIT_FAILURE);
    }
    const std::streamoff data0 = d.tellg();
    const uint64_t npts = (uint64_t)(fab.hi[0] - fab.lo[0] + 1) * (fab.hi[1] - fab.lo[1] + 1) *
                          (fab.hi[2] - fab.lo[2] + 1);
    for (size_t c = 0; c < comps.size(); ++c) {
        double* out = dst + c * npts;
        d.seekg(data0 + (std::streamoff)(8ull * npts * comps[c]));
        if (!d.read(reinterpret_cast<char*>(out), (std::streamsize)(8 * npts))) {
            log_error("Truncated FAB in " + fab.file);
            std::exit(EXIT_FAILURE);
        }
        if (fab.big_endian)
            for (uint64_t i = 0; i < npts; ++i) {
                uint64_t v;
                std::memcpy(&v, out + i, 8);
                v = __builtin_bswap64(v);
                std::memcpy(out + i, &v, 8);
            }
    }
}

}  // namespace wavelet_amd

using namespace wavelet_amd;

AllData preprocess_data(std::vector<std::string> files, std::vector<std::string> components,
                        std::vector<int> levels) {
    AllData ret;
    const size_t nc = components.size();
    ret.min_values.assign(nc, FLT_MAX);
    ret.max_values.assign(nc, FLT_MIN);  // FLT_MIN: the smallest positive float (reference quirk)
    for (size_t i = 0; i < files.size(); ++i) {
        const PlotHeader h = read_plot_header(files[i]);
        if (i == 0) {
            ret.comp_idxs = match_components(h, components);
            if (ret.comp_idxs.empty() && !components.empty()) {
                log_error("Some components you entered were not found. Check that the names you entered match "
                          "their names exactly in the AMReX Header files.");
                return {};
            }
            ret.amrexinfo.ref_ratios = h.ref_ratios;
        }
        if (h.dim != 3) log_error("Error: you are using a 3D build to open a " + std::to_string(h.dim) + "D plotfile");
        ret.amrexinfo.true_times.push_back(h.true_time);
        ret.amrexinfo.geomcellinfo.push_back(h.geomcell);
        ret.amrexinfo.xDim = h.xDim;
        ret.amrexinfo.yDim = h.yDim;
        ret.amrexinfo.zDim = h.zDim;
        std::vector<int> steps(levels.size(), 0);
        for (size_t l = 0; l < levels.size() && l < h.steps.size(); ++l) steps[l] = h.steps[l];
        ret.amrexinfo.level_steps.push_back(steps);

        std::vector<std::vector<multiBox3D>> fboxes;
        std::vector<std::vector<Location>> flocs;
        std::vector<std::vector<Dimensions>> fdims;
        std::vector<int> fcounts;
        for (int level : levels) {
            const std::vector<FabRef> fabs = read_level_index(files[i], level);
            std::vector<multiBox3D> boxes;
            std::vector<Location> locs;
            std::vector<Dimensions> dims;
            std::vector<float> lmin(nc, FLT_MAX), lmax(nc, FLT_MIN);
            std::vector<double> buf;
            for (const FabRef& f : fabs) {
                const int W = f.hi[0] - f.lo[0] + 1, H = f.hi[1] - f.lo[1] + 1, D = f.hi[2] - f.lo[2] + 1;
                const size_t npts = (size_t)W * H * D;
                locs.push_back({f.lo[0], f.lo[1], f.lo[2]});
                dims.push_back({W, H, D});
                buf.resize(npts * ret.comp_idxs.size());
                read_fab(f, ret.comp_idxs, buf.data());
                multiBox3D mb;
                for (size_t c = 0; c < ret.comp_idxs.size(); ++c) {
                    Box3D b(W, H, D, 0.0f);
                    float* o = b.data();
                    const double* s = buf.data() + c * npts;
                    for (size_t k = 0; k < npts; ++k) {
                        const float v = (float)s[k];  // src/preprocess.cpp:78
                        o[k] = v;
                        if (v < lmin[c]) lmin[c] = v;
                        if (v > lmax[c]) lmax[c] = v;
                    }
                    mb.push_back(std::move(b));
                }
                boxes.push_back(std::move(mb));
            }
            log_info("Processed data from time " + std::to_string(i) + ", level " + std::to_string(level));
            fcounts.push_back((int)fabs.size());
            fboxes.push_back(std::move(boxes));
            flocs.push_back(std::move(locs));
            fdims.push_back(std::move(dims));
            for (size_t c = 0; c < nc; ++c) {
                if (lmin[c] < ret.min_values[c]) ret.min_values[c] = lmin[c];
                if (lmax[c] > ret.max_values[c]) ret.max_values[c] = lmax[c];
            }
        }
        ret.boxes.push_back(std::move(fboxes));
        ret.locations.push_back(std::move(flocs));
        ret.dimensions.push_back(std::move(fdims));
        ret.box_counts.push_back(std::move(fcounts));
    }
    return ret;
}
