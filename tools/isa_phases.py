"""Static instruction counts of extract_kernel per source-line range (phase), from the gfx950 ISA
with line tables:  python tools/isa_phases.py [asm]  (default: builds /tmp/extract_g.s)."""
import collections, os, re, subprocess, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CS = os.path.join(R, "dsp-audioreclabs_amd", "csrc")
asm = sys.argv[1] if len(sys.argv) > 1 else "/tmp/extract_g.s"
if len(sys.argv) == 1:
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17", "-I" + os.path.join(R, "include"), "-I" + CS,
                    "--offload-device-only", "-gline-tables-only", "-S", os.path.join(CS, "extract.hip"), "-o", asm], check=True)
src = open(os.path.join(CS, "extract.hip")).read().split("\n")
body = ([i + 1 for i, l in enumerate(src) if "bool clip_body(" in l][0],
        [i + 1 for i, l in enumerate(src) if "void write_bad_clip(" in l][0])
marks = [(i + 1, l.strip()) for i, l in enumerate(src) if re.match(r"\s*// ---- R\d", l) or "STAMP(i," in l]
def phase(line):
    name = "pre"
    for ln, txt in marks:
        if ln <= line: name = "%d:%s" % (ln, txt[:50])
    return name
cur = None; fn = None
fidx = set()
for l in open(asm):
    m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]*)"', l) or re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"', l)
    if m and m.group(2).endswith("extract.hip"): fidx.add(m.group(1))
cnt = collections.defaultdict(collections.Counter)
for l in open(asm).read().split("\n"):
    m = re.match(r"^(_Z\S+):", l)
    if m: fn = m.group(1)
    m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
    if m:
        # innermost location of the inlining chain that lies inside clip_body
        chain = [int(x) for x in re.findall(r"extract\.hip:(\d+)", l)]
        inside = [x for x in chain if body[0] <= x <= body[1]]
        if inside: cur = inside[0]
        elif chain and chain[0] > 0: cur = chain[0]
    if fn and "extract_kernel" in fn and cur and re.match(r"\s+[vsd][a-z0-9_]+", l) and not l.strip().startswith("s_waitcnt"):
        op = l.split()[0]
        kind = "LDS" if op.startswith("ds_") else "VMEM" if op.startswith(("global_", "buffer_", "scratch_")) else "VALU" if op.startswith("v_") else "SALU"
        cnt[phase(cur)][kind] += 1
for k in sorted(cnt, key=lambda x: int(x.split(":")[0]) if x != "pre" else 0):
    c = cnt[k]; print("%-62s VALU %5d SALU %5d LDS %4d VMEM %4d" % (k, c["VALU"], c["SALU"], c["LDS"], c["VMEM"]))
