"""Build an experiment variant of the engine: libmr_engine_<name>.so with extra
-D flags (selected at run time with MR_ENGINE_LIB=<name>).
Usage: python scripts/build_variant.py NAME [-DFLAG ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from musicrecommendation_amd import build as b  # noqa: E402

name, flags = sys.argv[1], sys.argv[2:]
b._compile_all([(os.path.join(b.HERE, f"libmr_engine_{name}.so"), flags)], verbose=False)
print(name, flags)
