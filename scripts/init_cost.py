#!/usr/bin/env python3
"""Where the CLI's fixed cost goes (DESIGN.md "End-to-end"): HIP init + context creation,
index load, index upload (derived tables built on the device), per call of the native
library, timed in a fresh process.  Prints one JSON line.
  python scripts/init_cost.py INDEX_PREFIX"""
import json
import sys
import time

t0 = time.time()
sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
import ntcomp_amd as nt  # noqa: E402

nt.lib()
t1 = time.time()
c = nt.GpuContext(0)
t2 = time.time()
ix = nt.Index.load(sys.argv[1])
t3 = time.time()
c.upload(ix)
t4 = time.time()
up = {k: c.get_option(k) / 1e6 for k in ("upload_host_us", "upload_total_us")}
c2 = nt.GpuContext(0).share_index(c)
t5 = time.time()
c2.close()
c.close()
t6 = time.time()
print(json.dumps({"import_and_dlopen_s": round(t1 - t0, 3), "ctx_create_s": round(t2 - t1, 3),
                  "index_load_s": round(t3 - t2, 3), "upload_s": round(t4 - t3, 3),
                  "upload_host_derive_s": round(up["upload_host_us"], 3), "upload_total_s": round(up["upload_total_us"], 3),
                  "second_ctx_share_s": round(t5 - t4, 3), "close_s": round(t6 - t5, 3), "nodes": ix.n}))
