"""Code bytes of extract_kernel per phase (source-line range) for instruction-cache budgeting:
python tools/code_bytes.py [-Dmacro ...].  Pairs the .s (inlining chains -> phase) with the
disassembled code object (instruction sizes) in order."""
import collections, os, re, subprocess, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CS = os.path.join(R, "dsp-audioreclabs_amd", "csrc")
src_path = os.path.join(CS, "extract.hip")
flags = ["-O3", "--offload-arch=gfx950", "-std=c++17", "-I" + os.path.join(R, "include"), "-Wno-unused-function",
         "--offload-device-only", "-gline-tables-only"] + sys.argv[1:]
hip = "/opt/rocm/bin/hipcc"
KSEL = os.environ.get("KSEL", "extract_kernelILb1E")  # the fast instantiation
subprocess.run([hip] + flags + ["-S", src_path, "-o", "/tmp/cb.s"], check=True, stderr=subprocess.DEVNULL)
subprocess.run([hip] + flags + ["-c", src_path, "-o", "/tmp/cb.o"], check=True, stderr=subprocess.DEVNULL)
obj = "/tmp/cb.o"
if subprocess.run(["file", obj], capture_output=True, text=True).stdout.find("ELF") < 0:
    subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--unbundle", "--type=o", "--input=" + obj,
                    "--output=/tmp/cb.gpu.o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"], check=True)
    obj = "/tmp/cb.gpu.o"
dis = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", obj], capture_output=True, text=True).stdout
src = open(src_path).read().split("\n")
body = ([i + 1 for i, l in enumerate(src) if "bool clip_body(" in l][0],
        [i + 1 for i, l in enumerate(src) if "void write_bad_clip(" in l][0])
marks = [(i + 1, l.strip()) for i, l in enumerate(src) if re.match(r"\s*// ---- R\d", l) or "STAMP(i," in l]
def phase(line):
    name = "pre"
    for ln, txt in marks:
        if ln <= line: name = "%d:%s" % (ln, txt[:50])
    return name
# objdump: (mnemonic, size) of extract_kernel
ins = []
infn = False
for l in dis.split("\n"):
    m = re.match(r"^[0-9a-f]+ <(\S+)>:", l)
    if m: infn = KSEL in m.group(1); continue
    m = re.match(r"\s+(\S+).*//\s*([0-9A-F]+):((?:\s[0-9A-F]{8})+)", l)
    if infn and m: ins.append((m.group(1), 4 * len(m.group(3).split())))
# .s: (mnemonic, phase) of extract_kernel
sins = []
cur = None; fn = None
for l in open("/tmp/cb.s").read().split("\n"):
    m = re.match(r"^(_Z\S+):", l)
    if m: fn = m.group(1)
    if re.match(r"^\s*\.size\s", l): fn = None
    m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
    if m:
        chain = [int(x) for x in re.findall(r"extract\.hip:(\d+)", l)]
        inside = [x for x in chain if body[0] <= x <= body[1]]
        if inside: cur = inside[0]
        elif chain and chain[0] > 0: cur = chain[0]
    if fn and KSEL in fn and re.match(r"\s+[vsdgb][a-z0-9_]+(\s|$)", l) and not l.strip().startswith((".", ";")):
        sins.append((l.split()[0], phase(cur) if cur else "pre"))
n = min(len(ins), len(sins))
mism = sum(1 for a, b in zip(ins, sins) if a[0] != b[0])
tot = collections.Counter()
scr = collections.Counter()
rl = collections.Counter()
for (op, sz), (_, ph) in zip(ins, sins):
    tot[ph] += sz
    if op.startswith("scratch_"): scr[ph] += 1
    if op.startswith(("v_readlane", "v_writelane")): rl[ph] += 1
for k in sorted(tot, key=lambda x: int(x.split(":")[0]) if x != "pre" else 0):
    print("%-62s %6d B  scratch %3d  lane r/w %3d" % (k, tot[k], scr[k], rl[k]))
print("total %d B (objdump %d instrs, .s %d, mnemonic mismatches %d)" % (sum(sz for _, sz in ins), len(ins), len(sins), mism))
