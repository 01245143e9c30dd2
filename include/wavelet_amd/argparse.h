// argparse.h — run configuration and file/level selection
// (src/argparse.h:7-34, src/argparse.cpp).
//
// The reference reads its parameters through amrex::ParmParse, initialised
// from argv by amrex::Initialize.  Here init_params(argc, argv) plays that
// part; parameters use the same command-line syntax
// (`datadir=../data/ minfile=plt07400 ... components="Temp pressure" -c`).
#pragma once

#include <string>
#include <vector>

struct Config {
    std::string data_dir;
    std::string compressed_dir;
    std::string out_dir;
    std::string min_time, max_time;
    int min_level = 0, max_level = 0;
    float keep = 0.0f;
    std::vector<std::string> components;
    // Not a reference parameter: `xzpreset=N` (0-9, "Ne"
    // for the extreme variant) selects the xz preset of -c; default 6, the
    // reference's (src/compressor.cpp:261).  -1: not given ($WCAMD_XZ_PRESET or 6).
    int xz_preset = -1;
};

// Stand-in for amrex::Initialize's ParmParse setup: parse `name=value ...`
// definitions from argv (a definition's values run up to the next `name=`).
void init_params(int argc, char* argv[]);

Config parse_config_compress();    // datadir minfile maxfile minlevel maxlevel components keep compresseddir
Config parse_config_decompress();  // compresseddir out

bool has_flag(int argc, char* argv[], const std::string& flag);

// Digits of the name (all of them, leading zeros dropped) as an int; -1 if none.
int clean_string(std::string filename);

// Entries of data_dir whose clean_string lies in [clean(min), clean(max)], sorted by it.
std::vector<std::string> format_files(std::string data_dir, std::string min_time, std::string max_time);

std::vector<int> format_levels(int min_level, int max_level);
