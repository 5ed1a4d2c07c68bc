"""Per-kernel ISA report of a device assembly file (hipcc --offload-device-only -S):
VGPRs, scratch accesses and full vmcnt drains, for the kernels whose name matches a pattern.
Usage: python tools/isa_report.py file.s PATTERN [dump_name_substring out.s]"""
import re
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    lines = open(path).read().split('\n')
    heads = [i for i, l in enumerate(lines) if re.match(r'^_Z\S*:', l) and re.search(pat, l)]
    for i in heads:
        name = lines[i].split(':')[0]
        end = next(j for j in range(i, len(lines)) if lines[j].startswith('.Lfunc_end'))
        body = lines[i:end]
        vg = next((l.split(',')[-1].strip(' )') for l in lines if l.startswith('\t.set ' + name + '.num_vgpr')), '?')
        scr = sum('scratch_' in l for l in body)
        v0 = sum('vmcnt(0)' in l for l in body)
        mf = sum('v_mfma' in l for l in body)
        print(f'{name[:90]:90s} vgpr {vg:>4s} scratch {scr:4d} vmcnt0 {v0:3d} mfma {mf}')
        if len(sys.argv) > 4 and sys.argv[3] in name:
            open(sys.argv[4], 'w').write('\n'.join(body))


if __name__ == '__main__':
    main()
