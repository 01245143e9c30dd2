// tmpdir.h — scratch directory removed on destruction, as the reference's
// TempDir (src/tmpdir.h:7-36): mkdtemp under the system temp path.
#pragma once

#include <unistd.h>

#include <filesystem>
#include <string>

class TempDir {
public:
    TempDir() {
        std::string tmpl = (std::filesystem::temp_directory_path() / "wavelet_compress.XXXXXX").string();
        if (mkdtemp(tmpl.data())) path_ = tmpl;
    }
    TempDir(const TempDir&) = delete;
    TempDir& operator=(const TempDir&) = delete;
    ~TempDir() {
        std::error_code ec;
        if (!path_.empty()) std::filesystem::remove_all(path_, ec);
    }
    const std::filesystem::path& path() const { return path_; }

private:
    std::filesystem::path path_;
};
