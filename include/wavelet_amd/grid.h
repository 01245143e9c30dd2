// grid.h — dense 3-D grid with the reference's Grid3D<T> interface
// (src/grid.h:6-103): x-fastest storage `x + W*(y + H*z)`, bounds-checked
// access that throws std::out_of_range, move-only with an explicit clone().
// The C-ABI consumes the contiguous buffer through data() with no copy.
#pragma once

#include <cmath>
#include <cstddef>
#include <stdexcept>
#include <vector>

template <class T>
class Grid3D {
public:
    Grid3D() = default;
    Grid3D(size_t width, size_t height, size_t depth, T initial_value = T())
        : w_(width), h_(height), d_(depth), cells_(width * height * depth, initial_value) {}

    Grid3D(const Grid3D&) = delete;
    Grid3D& operator=(const Grid3D&) = delete;
    Grid3D(Grid3D&&) noexcept = default;
    Grid3D& operator=(Grid3D&&) noexcept = default;

    Grid3D clone() const {
        Grid3D g;
        g.w_ = w_;
        g.h_ = h_;
        g.d_ = d_;
        g.cells_ = cells_;
        return g;
    }

    bool is_valid() const { return cells_.size() == w_ * h_ * d_; }
    size_t data_size() const { return cells_.size(); }

    const T& get(size_t x, size_t y, size_t z) const { return cells_[offset(x, y, z)]; }
    void set(size_t x, size_t y, size_t z, T v) { cells_[offset(x, y, z)] = v; }
    T& operator()(size_t x, size_t y, size_t z) { return cells_[offset(x, y, z)]; }
    const T& operator()(size_t x, size_t y, size_t z) const { return cells_[offset(x, y, z)]; }

    size_t width() const { return w_; }
    size_t height() const { return h_; }
    size_t depth() const { return d_; }

    // z, y, x nesting like the reference's iterate(); f(value, x, y, z)
    template <class F>
    void iterate(F f) {
        for (size_t z = 0; z < d_; ++z)
            for (size_t y = 0; y < h_; ++y)
                for (size_t x = 0; x < w_; ++x) f(cells_[offset(x, y, z)], (int)x, (int)y, (int)z);
    }

    bool equals(const Grid3D<T>& o, float error) const {
        if (w_ != o.w_ || h_ != o.h_ || d_ != o.d_) return false;
        for (size_t i = 0; i < cells_.size(); ++i)
            if (std::abs(cells_[i] - o.cells_[i]) > error) return false;
        return true;
    }

    // Contiguous storage for the GPU boundary (no counterpart in the reference).
    T* data() { return cells_.data(); }
    const T* data() const { return cells_.data(); }

private:
    size_t offset(size_t x, size_t y, size_t z) const {
        if (x >= w_ || y >= h_ || z >= d_) throw std::out_of_range("Grid3D index out of range");
        return x + w_ * (y + h_ * z);
    }

    size_t w_ = 0, h_ = 0, d_ = 0;
    std::vector<T> cells_;
};
