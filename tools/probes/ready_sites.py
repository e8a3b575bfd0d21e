"""Which call sites make the compute stream wait for the whole staged update (FlatParamStore.params_ready)
during a bench run:  python tools/probes/ready_sites.py <bench args>"""
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hetseq_amd.runtime import flat  # noqa: E402

SITES = collections.Counter()
_orig = flat.FlatParamStore.params_ready


def params_ready(self, *a, **k):
    st = traceback.extract_stack(limit=6)[:-1]
    SITES[" <- ".join("%s:%d %s" % (os.path.basename(f.filename), f.lineno, f.name) for f in reversed(st))] += 1
    return _orig(self, *a, **k)


flat.FlatParamStore.params_ready = params_ready
import bench  # noqa: E402

sys.argv = ["bench.py"] + sys.argv[1:]
rc = bench.main()
for s, n in SITES.most_common():
    print("%5d  %s" % (n, s))
sys.exit(rc)
