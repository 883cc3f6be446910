"""MI355X-native path-tracing core for sourcedennis/wasm-pathtracer's hot path.

The product is libwpt.so (HIP kernels for gfx950 + the C ABI of
include/wpt.h). This package only binds it (``_lib``), mirrors the reference's
``wasm_interface.rs`` operator surface (``interface``) and provides the
JavaScript-side scene inputs (``scenes``).
"""
from . import interface, scenes  # noqa: F401
from ._lib import lib  # noqa: F401
