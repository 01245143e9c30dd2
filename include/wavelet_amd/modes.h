// modes.h — the reference's run modes (src/modes.h, src/modes.cpp): -c, -d,
// -estimate, batched over all units of a run on the GPU with the xz stage on a
// host thread pool.
#pragma once

#include "argparse.h"

int compress(const Config& cfg);
int decompress(const Config& cfg);
int estimate(Config& cfg);
