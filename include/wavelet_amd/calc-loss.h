// calc-loss.h — drop-in for the reference's src/calc-loss.h:6-16.
#pragma once

#include "box-structs.h"

// Per-component RMSE of one box (GPU, src/calc-loss.cpp:12-43).
std::vector<double> calc_rmse_per_box(const multiBox3D& actual, const multiBox3D& pred, int num_components);

double calc_adj_loss(double rmse, double range);

double calc_size(std::string path);
