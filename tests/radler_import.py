"""Import the product's `radler` pybind11 module from the in-tree build."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ska-sdp-func-radler_amd")
if PKG not in sys.path:
    sys.path.insert(0, PKG)

import radler  # noqa: E402,F401
