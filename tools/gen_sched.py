"""Generate the IB fast path's per-degree fold schedules (csrc/ib_sched.inc).

The check-node (variable-node) update of one group of S codewords is a DAG of lookup chains
(kernels_template_irreg.cl:205-231 / :151-160, prefix-shared as in ib_kernels.hip):
  CN degree D:  out0 chain  in1 -> B0(.,in2) -> ... -> B_{D-3}(.,in_{D-1})           (D-2 steps)
                P chain     in0 -> B0(.,in1) = P2 -> B1(.,in2) = P3 ... -> out_{D-1}  (D-2 steps)
                chain w     P_w -> B_{w-1}(.,in_{w+1}) -> ... -> out_w, w=1..D-2     (D-1-w steps)
  VN degree D:  out0 chain  V0(c,in1) -> V1(.,in2) -> ... -> out0                    (D-1 steps)
                Q chain     V0(c,in0) = Q1 -> V1(.,in1) = Q2 ... -> out_{D-1}        (D-1 steps)
                chain w     Q_w -> V_w(.,in_{w+1}) -> ... -> out_w, w=1..D-2         (D-1-w steps)
Every chain is a sequence of dependent LDS lookups; chains are independent once their start value
exists, so the critical path is D-2 (CN) / D-1 (VN) steps, not the 25 / 35 of running them one
after another. This script list-schedules the chains onto L concurrent lanes (critical path first)
and emits straight-line code with one SSA name per value (no register copies): each time step
issues the lookups of every running lane for all S sub-slots back to back.

Column fetches. Input in_j meets the SAME table in every chain that did not fold it into its
prefix: B_{j-2}(., in_j) in the out0 chain and in chains w = 1..j-1 of a check node (j uses),
V_{j-1}(., in_j) likewise for a variable node. For the last NC inputs of a node (cn_ncols(D) /
vn_ncols(D) in common.h) the kernel reads that table's whole column T(., m = in_j) once - 16
nibbles, one conflict-free ds_read_b64 of a bank-replicated column image - and selects entry t
with a 64-bit shift by 4t (csel). Those j lookups then cost one LDS read instead of j (DVB-S2
degree-7 check: 25 LDS reads -> 16; degree-8 variable: 35 -> 20), paid with one extra VALU per
lookup; the LDS array, not VALU issue, is what bounds the byte-lookup kernels. Column steps come
last in every chain (the NC inputs are the last ones folded), so a byte lookup never follows one.

Measured (tools/variants.py nc23/nc22/nc33/s2, DVB-S2 B=8192 i_max=50): column fetches LOSE - CN
0.464 -> 0.622 ms, VN 0.478 -> 0.526 ms at NC = 2/3 (170.9k -> 140.9k cw/s). The 64-bit shift and the
nibble masks cost more VALU issue than the saved LDS reads return, so the default is NC = 0 (no
column images, the byte-lookup schedules of before); the option stays for other code profiles.

usage: python tools/gen_sched.py [S_cn L_cn S_vn L_vn [NC_cn NC_vn]] > informationbottleneckdecodingldpc_amd/csrc/ib_sched.inc
(measured on DVB-S2: CN S=4 L=2, VN S=2 L=4, NC 0 0; NC_cn / NC_vn must equal IBL_NC_CN / IBL_NC_VN
of the build that includes the file - the file static_asserts it)
"""
import sys

KMAXD = 16


def slot_off(l):   # csrc/common.h: quad l >> 2 in super-region l >> 3, half (l >> 2) & 1, byte l & 3
    return (l >> 3) * 65536 + ((l >> 2) & 1) * 128 + (l & 3)


def cn_ncols(D, nc):
    return nc if 5 <= D <= 8 else 0


def vn_ncols(D, nc):
    return nc if 6 <= D <= 8 else 0


def cn_chains(D):
    def st(j, l):
        sl = "0u" if j == D - 1 else ("fbase" if l == D - 3 else f"{slot_off(l)}u")
        return ("q", j, sl, l)
    ch = [dict(id="o0", start=("nib", 1), steps=[st(j, j - 2) for j in range(2, D)], out=0),
          dict(id="P", start=("nib", 0), steps=[st(w, w - 1) for w in range(1, D - 1)], out=D - 1)]
    for w in range(1, D - 1):
        s0 = ("nib", 0) if w == 1 else ("val", "P", w - 2)              # P_w = P chain after step w-2
        ch.append(dict(id=f"c{w}", start=s0, steps=[st(j, j - 2) for j in range(w + 1, D)], out=w))
    return ch


def vn_chains(D):
    def st(op, j, l):
        sl = "0u" if j == D - 1 else ("fbase" if l == D - 2 else f"{slot_off(l)}u")
        return (op, j, sl, l)
    ch = [dict(id="o0", start=("chan",), steps=[st("c", 1, 0)] + [st("q", j, j - 1) for j in range(2, D)], out=0),
          dict(id="Q", start=("chan",), steps=[st("c", 0, 0)] + [st("q", w, w) for w in range(1, D - 1)], out=D - 1)]
    for w in range(1, D - 1):
        ch.append(dict(id=f"c{w}", start=("val", "Q", w - 1),           # Q_w = Q chain after step w-1
                       steps=[st("q", j, j - 1) for j in range(w + 1, D)], out=w))
    return ch


def schedule(chains, L):
    """List scheduling: returns [(time, [(chain, step_index), ...]), ...]."""
    by_id = {c["id"]: c for c in chains}
    # downstream weight: a prefix chain gates every suffix chain -> schedule it first
    for c in chains:
        c["prio"] = len(c["steps"]) + (100 if c["id"] in ("P", "Q") else 0)
    ready_at = {}
    for c in chains:
        ready_at[c["id"]] = 0 if c["start"][0] in ("nib", "chan") else None
    running = []     # [chain_id, next_step]
    pending = [c["id"] for c in chains]
    out = []
    t = 0
    while pending or running:
        cand = [cid for cid in pending if ready_at[cid] is not None and ready_at[cid] <= t]
        cand.sort(key=lambda cid: (-by_id[cid]["prio"], chains.index(by_id[cid])))
        while len(running) < L and cand:
            cid = cand.pop(0)
            pending.remove(cid)
            running.append([cid, 0])
        if not running:
            raise RuntimeError("deadlock")
        issued = []
        for r in running:
            issued.append((r[0], r[1]))
            r[1] += 1
        out.append((t, issued))
        # exports become available next step
        for cid, k in issued:
            for c in chains:
                st = c["start"]
                if st[0] == "val" and st[1] == cid and st[2] == k:
                    ready_at[c["id"]] = t + 1
        running = [r for r in running if r[1] < len(by_id[r[0]]["steps"])]
        t += 1
    return out


def emit_body(kind, D, S, L, NC):
    chains = cn_chains(D) if kind == "cn" else vn_chains(D)
    by_id = {c["id"]: c for c in chains}
    sched = schedule(chains, L)
    back = 2 if kind == "cn" else 1          # input j meets table j-back in every non-prefix chain

    def is_col(step):
        op, j, _, l = step
        return op == "q" and j >= D - NC and l == j - back

    for c in chains:   # column steps are the tail of every chain
        cols = [is_col(s) for s in c["steps"]]
        assert cols == sorted(cols), (kind, D, c["id"])
    lines = []
    u8_in = sorted({s[1] for c in chains for s in c["steps"] if not is_col(s)})
    col_in = sorted({s[1] for c in chains for s in c["steps"] if is_col(s)})
    if D - 1 in u8_in:   # column base of the last input: final-table slot added once, not per codeword
        lines.append("  const uint32_t lane4f = lane4 + fbase;")
    for j in u8_in:
        for s in range(S):
            base = "lane4f" if j == D - 1 else "lane4"
            lines.append(f"  const uint32_t q{j}_{s} = colq(in[{j}], k0 + {s}, {base});")
    for j in col_in:
        for s in range(S):
            lines.append(f"  const uint64_t C{j}_{s} = colf(nib(in[{j}], k0 + {s}), cb[{j - (D - NC)}]);")
    if kind == "vn":   # channel nibble as a row term: luc merges it with a column term in one v_lshl_or
        for s in range(S):
            lines.append(f"  const uint32_t c_{s} = nib(chw, k0 + {s});")

    def name(cid, k, s):
        return f"v_{cid}_{k}_{s}"

    def start_val(c, s):
        st = c["start"]
        if st[0] == "nib":
            return f"nib(in[{st[1]}], k0 + {s})"
        if st[0] == "val":
            return name(st[1], st[2], s)
        raise AssertionError

    for t, issued in sched:
        lines.append(f"  // step {t}: " + ", ".join(f"{cid}[{k}]" for cid, k in issued))
        for cid, k in issued:
            c = by_id[cid]
            step = c["steps"][k]
            op, j, sl, _ = step
            for s in range(S):
                if op == "c":
                    expr = f"luc(c_{s}, q{j}_{s}, {sl})"
                else:
                    prev = start_val(c, s) if k == 0 else name(cid, k - 1, s)
                    expr = f"csel(C{j}_{s}, {prev} << 2)" if is_col(step) else f"luc({prev}, q{j}_{s}, {sl})"
                lines.append(f"  const uint32_t {name(cid, k, s)} = {expr};")
        for cid, k in issued:
            c = by_id[cid]
            if k == len(c["steps"]) - 1:
                col = is_col(c["steps"][k])
                vals = [f"({name(cid, k, s)} & 15u)" if col else name(cid, k, s) for s in range(S)]
                pk = vals[0]
                for s in range(1, S):
                    pk = f"{pk} | ({vals[s]} << {4 * s})"
                lines.append(f"  o[{c['out']}] |= ({pk}) << (4 * k0);")
    return lines


def main():
    """args: S_cn L_cn [S_vn L_vn [NC_cn NC_vn]] (group size and chain lanes per kernel, for degrees
    <= 8; larger degrees use S = 2, L = 4 so the MAXD = 16 bodies keep their occupancy; column-fetched
    trailing inputs per check / variable node)."""
    a = [int(x) for x in sys.argv[1:]] or [4, 2, 2, 4]
    Sc, Lc = a[0], a[1]
    Sv, Lv = (a[2], a[3]) if len(a) >= 4 else (Sc, Lc)
    NCc, NCv = (a[4], a[5]) if len(a) >= 6 else (0, 0)

    def cfg(S, L, D):
        return (S, L) if D <= 8 else (2, 4)
    print(f"// GENERATED by tools/gen_sched.py {' '.join(sys.argv[1:])} -- do not edit.")
    print(f"// Fold schedules of the IB fast path (degrees <= 8): CN groups of {Sc} codewords with up to {Lc}")
    print(f"// chains in flight, VN groups of {Sv} codewords with up to {Lv}; degrees > 8: 2 codewords, 4 chains.")
    print(f"// Column fetches: the last {NCc} inputs of checks of degree 5..8, the last {NCv} of variables of degree 6..8.")
    print(f"static_assert(cn_ncols(7) == {cn_ncols(7, NCc)} && vn_ncols(8) == {vn_ncols(8, NCv)},")
    print("              \"ib_sched.inc was generated for other IBL_NC_CN / IBL_NC_VN\");")
    print(f"__host__ __device__ constexpr int cn_sched_s(int D) {{ return D <= 8 ? {Sc} : 2; }}")
    print(f"__host__ __device__ constexpr int vn_sched_s(int D) {{ return D <= 8 ? {Sv} : 2; }}")
    print("template <int D> __device__ __forceinline__ void cn_group(uint32_t lane4, const uint32_t (&in)[D],")
    print("                                                         uint32_t fbase, const uint32_t (&cb)[4],")
    print("                                                         uint32_t (&o)[D], int k0);")
    print("template <int D> __device__ __forceinline__ void vn_group(uint32_t lane4, const uint32_t (&in)[D],")
    print("                                                         uint32_t chw, uint32_t fbase, const uint32_t (&cb)[4],")
    print("                                                         uint32_t (&o)[D], int k0);")
    for D in range(3, KMAXD + 1):
        print(f"template <> __device__ __forceinline__ void cn_group<{D}>(uint32_t lane4, const uint32_t (&in)[{D}],")
        print("                                                         uint32_t fbase, const uint32_t (&cb)[4],")
        print(f"                                                         uint32_t (&o)[{D}], int k0) {{")
        print("\n".join(emit_body("cn", D, *cfg(Sc, Lc, D), cn_ncols(D, NCc))))
        print("}")
    for D in range(2, KMAXD + 1):
        print(f"template <> __device__ __forceinline__ void vn_group<{D}>(uint32_t lane4, const uint32_t (&in)[{D}],")
        print("                                                         uint32_t chw, uint32_t fbase, const uint32_t (&cb)[4],")
        print(f"                                                         uint32_t (&o)[{D}], int k0) {{")
        print("\n".join(emit_body("vn", D, *cfg(Sv, Lv, D), vn_ncols(D, NCv))))
        print("}")


if __name__ == "__main__":
    main()
