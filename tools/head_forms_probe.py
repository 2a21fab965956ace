"""Which head-kernel form changes the bits: 3 S3 split2h steps per env in fresh processes, digests of
each output (logs, each parameter / moment array, stream states).  usage: python tools/head_forms_probe.py"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = """
import hashlib, sys
sys.path.insert(0, %r); sys.path.insert(0, %r)
import numpy as np
import test_gpu_fullbatch as t
a = t._device_steps(50, 50, 2048, 3, 3, 0)
names = ["actor", "critic", "critic_target", "log_alpha", "actor_mu", "actor_nu", "critic_mu", "critic_nu"]
print("logs", {k: float(v) for k, v in sorted(a[0].items())})
for n, x in zip(names, a[1]):
    print(n, hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest()[:16])
""" % (ROOT, os.path.join(ROOT, "tests"))
for extra in ({}, {"MTSAC_HEAD_RW": "1"}, {"MTSAC_HEAD_RW": "2"}, {"MTSAC_HEAD_RW": "4"}):
    r = subprocess.run([sys.executable, "-c", CHILD], capture_output=True, text=True, env=dict(os.environ, **extra),
                       timeout=300)
    print("==", extra, "rc", r.returncode, flush=True)
    print(r.stdout[-3000:], r.stderr[-1500:] if r.returncode else "", flush=True)
