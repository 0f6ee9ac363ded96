"""Kernel time of one config-2 batch vs the LDS requested per workgroup
(DEPPY_LDS_PAD_KB, a diagnostic knob of the runtime): how residency per CU
maps to step time.  Run on the GPU box; one child process per setting."""
import json
import os
import subprocess
import sys

if len(sys.argv) > 1:
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import numpy as np
    from deppy_amd import _lib
    from tests.gpu_common import lowered_config
    lw = lowered_config(2, 10000, 1000)
    ctx = _lib.Context(0, 1)
    r = ctx.upload(lw.rec_off, lw.rec)
    for _ in range(3):
        r.run()
    ms = []
    for _ in range(10):
        r.run()
        ms.append(ctx.last_kernel_ms())
    print(json.dumps({"pad_kb": int(sys.argv[1]), "kernel_ms": float(np.median(ms))}), flush=True)
else:
    for pad in [0, 20, 24, 32, 40, 54, 80]:
        env = dict(os.environ, DEPPY_LDS_PAD_KB=str(pad))
        subprocess.run([sys.executable, __file__, str(pad)], env=env, check=True, timeout=120)
