// calc-loss.cpp — C++ mirror of src/calc-loss.cpp:12-65.
#include <filesystem>
#include <vector>

#include "host_ctx.h"
#include "wavelet_amd/calc-loss.h"

using namespace wavelet_amd;

std::vector<double> calc_rmse_per_box(const multiBox3D& actual, const multiBox3D& pred, int num_components) {
    std::vector<double> rmse(num_components > 0 ? num_components : 0, 0.0);
    if (num_components <= 0) return rmse;
    // Like the reference, every component is measured over actual[0]'s dims.
    const int W = (int)actual[0].width(), H = (int)actual[0].height(), D = (int)actual[0].depth();
    const uint64_t per = (uint64_t)W * H * D;
    std::vector<wc_unit> units(num_components);
    std::vector<float> a(per * num_components), p(per * num_components);
    for (int c = 0; c < num_components; ++c) {
        units[c] = wc_unit{per * c, W, H, D, 0};
        if (actual[c].data_size() < per || pred[c].data_size() < per) fatal("calc_rmse_per_box: box smaller than actual[0]");
        std::copy(actual[c].data(), actual[c].data() + per, a.begin() + per * c);
        std::copy(pred[c].data(), pred[c].data() + per, p.begin() + per * c);
    }
    wc_ctx* ctx = thread_ctx();
    check(ctx, wc_rmse_host(ctx, a.data(), WC_F32, p.data(), units.data(), num_components, rmse.data()), "GPU RMSE");
    return rmse;
}

double calc_adj_loss(double rmse, double range) { return rmse / range; }

double calc_size(std::string path) {
    double size = 0;
    for (const auto& e : std::filesystem::recursive_directory_iterator(path))
        if (e.is_regular_file()) size += (double)std::filesystem::file_size(e);
    return size;
}
