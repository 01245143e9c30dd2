"""Import shim for the `wavelet-compression_amd/` package.

The package directory keeps the project's name, which is not a valid Python
identifier; this module loads it under the name `wavelet_compression_amd` and
re-exports it, so `import wcamd` works from the repo root.
"""
import importlib.util
import sys
from pathlib import Path

_PKG_DIR = Path(__file__).resolve().parent / "wavelet-compression_amd"
_NAME = "wavelet_compression_amd"

if _NAME in sys.modules:
    _mod = sys.modules[_NAME]
else:
    _spec = importlib.util.spec_from_file_location(
        _NAME, _PKG_DIR / "__init__.py", submodule_search_locations=[str(_PKG_DIR)])
    _mod = importlib.util.module_from_spec(_spec)
    sys.modules[_NAME] = _mod
    _spec.loader.exec_module(_mod)

globals().update({k: v for k, v in vars(_mod).items() if not k.startswith("__")})
PACKAGE = _mod
PACKAGE_DIR = _PKG_DIR
