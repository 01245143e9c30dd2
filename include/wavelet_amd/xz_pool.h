// xz_pool.h — the xz stage of compress()/decompress() (src/compressor.cpp:256-291,
// src/decompressor.cpp:164-234) over a pool of host threads: one independent
// .xz stream per unit, so units encode and decode in parallel.
#pragma once

#include <cstddef>
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

namespace wavelet_amd {

// Threads for host stages: $WCAMD_THREADS, else $OMP_NUM_THREADS, else the core count.
int host_threads();

// Run fn(i) for i in [0, n) on `threads` threads (dynamic assignment).
void parallel_for(size_t n, int threads, const std::function<void(size_t)>& fn);

struct XzJob {
    const uint8_t* data;  // serialized payload
    size_t size;
    std::string path;     // output file
};

// The xz preset of every encoder in the process (an
// optional faster preset).  Default 6 = the reference's lzma_easy_encoder(6,
// CRC64) (src/compressor.cpp:261-262), byte-identical to its files; $WCAMD_XZ_PRESET
// or set_xz_preset() (the CLI's `xzpreset=`) select another.  Any preset is
// read back by the reference's lzma_stream_decoder(UINT64_MAX, LZMA_CONCATENATED)
// (src/decompressor.cpp:189), which takes the filter chain from the stream.
// A preset value is 0-9, optionally | LZMA_PRESET_EXTREME ("6e").
uint32_t xz_preset();
void set_xz_preset(uint32_t preset);
// "0".."9" with an optional trailing 'e' -> preset value; -1 if malformed.
int parse_xz_preset(const char* text);

// Encode each job (the current preset, CRC64) and write its file.  A
// file that cannot be opened is skipped (src/compressor.cpp:256-257); encoder
// failures exit.  Returns the bytes written.
uint64_t xz_write_files(const std::vector<XzJob>& jobs, int threads);

// Read and decode each file (stream decoder, concatenated streams).  Failures exit.
std::vector<std::string> xz_read_files(const std::vector<std::string>& paths, int threads);

// One buffer -> one .xz stream (preset xz_preset(), or `preset` when >= 0; CRC64).
std::string xz_encode(const uint8_t* data, size_t size, int preset = -1);
// The same without exiting: false and a message on an encoder failure.
bool xz_encode_try(const uint8_t* data, size_t size, std::string& out, const char*& err, int preset = -1);

// Opt-in write-behind of compress()'s files ($WCAMD_WRITE_BEHIND=1 or
// set_write_behind(true); default off = the reference's behaviour, every file
// written before compress() returns).  On: compress() queues each component's
// payload and returns; host_threads() workers encode and write the files.
// They are complete once flush_writes() returns, before decompress() reads one
// (flush_writes(path): that file's pending writes only), and at normal process exit.  set_write_behind(false) flushes first.  An encoder
// failure in a worker is reported (log + exit(EXIT_FAILURE), as compress()
// would) by the next flush, or at exit.
bool write_behind();
void set_write_behind(bool on);
void write_behind_submit(std::string payload, std::string path);
void note_write_behind_used();
void flush_writes();
void flush_writes(const std::string& path);

}  // namespace wavelet_amd
