// readandwrite.h — the run's side files (src/readandwrite.h): runinfo.raw,
// locations.raw, dimensions.raw, boxcounts.raw, amrexinfo.raw, byte-compatible
// with the reference's (native-endian; size_t-prefixed strings and vectors;
// locations/dimensions/box counts stored as float32; long double as 16 bytes).
#pragma once

#include <string>
#include <vector>

#include "box-structs.h"
#include "iterator.h"

void write_loc_dim_to_bin(LocDimData data, std::string path, std::string out_file, AMRIterator iterator);
LocDimData read_loc_dim_from_bin(std::string const& path, std::string const& in_file,
                                 std::vector<std::vector<int>> counts, AMRIterator iterator, int num_times,
                                 int num_levels);

void write_box_counts(std::vector<std::vector<int>> counts, std::string const& path, std::string const& out_file,
                      int num_times, int num_levels);
std::vector<std::vector<int>> read_box_counts(std::string path, std::string in_file, int num_times,
                                              int num_levels);

void write_amrexinfo(AMReXInfo info, std::string path, std::string out_file);
AMReXInfo read_amrex_info(std::string path, std::string in_file);

void write_runinfo(RunInfo info, std::string path, std::string out_file);
RunInfo read_runinfo(std::string path, std::string in_file);
