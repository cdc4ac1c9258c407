"""`src` — import name of the MI355X-native Mini-Petals framework.

The reference is launched as ``python -m src.main ...`` (reference src/main.py:775-838),
so the framework keeps ``src`` as its import name.  The implementation lives in the
package directory ``global_capstone_design_distributed-inference-of-llms-over-the-internet_amd/``
(a hyphenated, non-importable directory name); this module makes that directory the
package's search path, so ``src.main``, ``src.rpc_handler``, ``src.ops`` ... resolve there.
"""
import os as _os

PACKAGE_DIR = _os.path.join(
    _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
    "global_capstone_design_distributed-inference-of-llms-over-the-internet_amd",
)
__path__ = [PACKAGE_DIR]  # noqa: F811  (package search path -> implementation directory)
__version__ = "0.1.0"
