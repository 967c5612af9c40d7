"""Developer A/B helper: build libvst_hip with extra -D defines into _build/variants/<name>.so.
Usage: python tools/build_variant.py NAME DEF1=V DEF2=V ...; run with VST_LIB_VARIANT=<path>."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gbvst  # noqa: E402

name, defs = sys.argv[1], sys.argv[2:]
out = os.path.join(gbvst._lib.BUILD, "variants", "lib_%s.so" % name)
os.makedirs(os.path.dirname(out), exist_ok=True)
print(gbvst._lib.build(force=True, out=out, defines=list(defs) + ["VST_DEV_VARIANT=1"]))
