// iterator.h — the reference's AMRIterator (src/iterator.h:5-34): visits every
// (time, level, box) of a run in t-major, then level, then box order.
#pragma once

#include <cstddef>
#include <vector>

class AMRIterator {
public:
    AMRIterator(size_t num_times, size_t num_levels, const std::vector<std::vector<int>>& box_counts,
                size_t num_components)
        : nt_(num_times), nl_(num_levels), counts_(box_counts), nc_(num_components) {}

    template <class F>
    void iterate(F f) {
        for (int t = 0; t < (int)nt_; ++t)
            for (int l = 0; l < (int)nl_; ++l)
                for (int b = 0; b < counts_[t][l]; ++b) f(t, l, b);
    }

    size_t num_components() const { return nc_; }

private:
    size_t nt_, nl_;
    const std::vector<std::vector<int>>& counts_;
    size_t nc_;
};
