import sys, os, subprocess, gzip
REPO = os.getcwd()
code = r'''
import sys, os, gzip, faulthandler
faulthandler.enable()
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np, ntcomp_amd as nt
from test_cli import _bgzf_member
name, bpb, hp = sys.argv[1], int(sys.argv[2]), sys.argv[3] == "1"
genome = nt.synth_genome(31, 100_000)
ix = nt.Index.build([genome.tobytes()], 31)
ctx = nt.GpuContext(0); ctx.upload(ix)
n, L = 5 * 65536 + 999, 75
body = nt.synth_reads(genome, 32, 0, n, L, 10_000).reshape(n, L)
recs = [b"@r%d\n" % i + body[i].tobytes() + b"\n+\n" + b"F" * L + b"\n" for i in range(n)]
plain = b"".join(recs)
files = {"plain": plain, "crlf": plain.replace(b"\n", b"\r\n"),
         "mid_blank": b"".join(recs[:4 * 65536 + 5]) + b"\n" + b"".join(recs[4 * 65536 + 5:]),
         "plain_gz": gzip.compress(plain, 1),
         "plain_bgzf": b"".join(_bgzf_member(plain[i:i + 65000]) for i in range(0, len(plain), 65000))}
open("/tmp/d.fq", "wb").write(files[name])
fd = os.open("/tmp/d.dat", os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
st = nt.encode_file([ctx], "/tmp/d.fq", fd, blocks_per_batch=bpb, host_parse=hp)
os.close(fd)
print(name, bpb, hp, st["reads"], st["gpu_parsed"], flush=True)
'''
open("/tmp/diag_one.py", "w").write(code)
for name in ("plain", "crlf", "mid_blank", "plain_gz", "plain_bgzf"):
    for bpb in (1, 4):
        for hp in ("0", "1"):
            r = subprocess.run([sys.executable, "/tmp/diag_one.py", name, str(bpb), hp], capture_output=True, text=True, timeout=120)
            print(name, bpb, hp, "rc", r.returncode, r.stdout.strip()[-200:], r.stderr.strip()[-600:] if r.returncode else "", flush=True)
            if r.returncode < 0 or r.returncode > 1:
                sys.exit(0)
