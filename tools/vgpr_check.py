import sys, os, tempfile, subprocess, re
sys.path.insert(0, '.')
os.environ["RTN_DEBUG"] = "1"
from pathlib import Path
import bench
from retina_amd import pc
pc._LIB_PATH = pc._LIB_PATH.with_name("libretina_pc_exp.so")
for cfg in ("cfg3", "cfg4"):
    p = pc.Program.from_spec(bench.spec_for(cfg))
    co = p.code_object()
    d = tempfile.mkdtemp(); f = Path(d) / "k.co"; f.write_bytes(co)
    notes = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", str(f)], capture_output=True, text=True).stdout
    for blk in notes.split("  - .agpr_count")[1:]:
        g = dict(re.findall(r"\.(\w+):\s+(\S+)", blk))
        if g.get("name") == "rtn_pc_kernel_splitc":
            print(cfg, "notes vgpr_count", g.get("vgpr_count"), flush=True)
    ctx = pc.PacketContinue(p, 0)
    sys.stderr.flush()
