"""Search the query -> lane order of attn_tbl_kernel's bias-quad reads (csrc/attention.hip,
kAttnQmap): gfx950 ds_read_b128 serves 16-lane groups {0-3,12-15,20-27}, ...; a group is
conflict-free when its 16 table slots differ mod 16.  Prints the conflict count of the identity
order and of an annealed permutation, and writes the permutation (comma-separated) to the path
given as argv[1] (default /tmp/qperm.txt).  Developer tool."""
import math
import random
import sys

TBLN = 547
GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
GROUPS += [[l + 32 for l in g] for g in GROUPS]


def slot(q, g4):
    qz, qy, qx = q >> 6, (q >> 3) & 7, q & 7
    return (TBLN - 1) - ((qz + 7) * 23 + (qy + 7) * 15 + (qx + 7)) + ((g4 >> 1) * 15 + 4 * (g4 & 1))


def sub_cost(p, u):
    tot = 0
    for grp in GROUPS:
        cnt = {}
        for lane in grp:
            s = slot(p[u * 16 + (lane & 15)], lane >> 4) % 16
            cnt[s] = cnt.get(s, 0) + 1
        tot += sum(c * (c - 1) // 2 for c in cnt.values())  # colliding lane pairs
    return tot


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "/tmp/qperm.txt"
    random.seed(1)
    perm = list(range(512))
    print("identity order: colliding lane pairs", sum(sub_cost(perm, u) for u in range(32)))
    costs = [sub_cost(perm, u) for u in range(32)]
    total, temp = sum(costs), 2.0
    for _ in range(400000):
        i, j = random.randrange(512), random.randrange(512)
        ui, uj = i // 16, j // 16
        perm[i], perm[j] = perm[j], perm[i]
        ci = sub_cost(perm, ui)
        cj = sub_cost(perm, uj) if uj != ui else ci
        new = total - costs[ui] - (costs[uj] if uj != ui else 0) + ci + (cj if uj != ui else 0)
        if new <= total or random.random() < math.exp((total - new) / temp):
            costs[ui], costs[uj], total = ci, cj, new
        else:
            perm[i], perm[j] = perm[j], perm[i]
        temp = max(0.01, temp * 0.99998)
        if total == 0:
            break
    print("annealed order: colliding lane pairs", total)
    open(out, "w").write(",".join(map(str, perm)))


if __name__ == "__main__":
    main()
