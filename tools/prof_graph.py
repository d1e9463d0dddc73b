"""CPU profile of the create_mega_reads graph code (overlap_graph.cpp) on C2
records: the oracle aligns the first N C2 reads with create_mega_reads' flags
(-f, production -B / --max-count / --stretch-cap), the records go to
og_driver's RECORDS file, and og_driver times ReadGraph::process.
  python tools/prof_graph.py [N] [outdir]"""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    d = sys.argv[2] if len(sys.argv) > 2 else "/tmp/prof_graph"
    os.makedirs(d, exist_ok=True)
    from oracle import oracle as O
    from oracle import mega_reads as MR
    from tests.test_mega_reads import records_text
    from tools.synth import Dataset
    rf = os.path.join(d, "records")
    if not os.path.exists(rf):
        ds = Dataset("C2", seed=42, threads=8, n_pb=n)
        ul = [int(x) for x in ds.unitig_lengths]
        with open(os.path.join(d, "ul.txt"), "w") as f:
            f.writelines(f"{i} {x}\n" for i, x in enumerate(ul))
        t = time.time()
        oix = O.OracleIndex.from_records(ds.sr_names(), ds.sr_seqs(), 17)
        p = O.params(k=17, forward=True, unitigs_k=31, unitig_lengths=ul, bases_matching=15.0, max_count=5000,
                     stretch_cap=10000.0, psa_min=13)
        reads = [(nm.decode(), MR.records_of(oix, p, s)) for nm, s in zip(ds.pb_names(), ds.pb_seqs())]
        print(f"oracle records: {time.time() - t:.1f}s, {sum(len(r) for _, r in reads)} records", file=sys.stderr)
        with open(rf, "w") as f:
            f.write(records_text(reads))
    with open(os.path.join(d, "params"), "w") as f:
        f.write(f"31 1.3 3.0 0 0.029 100.0 greedy none {os.path.join(d, 'ul.txt')} -\n")
    exe = os.path.join(d, "og_driver")
    flags = os.environ.get("OG_FLAGS", "-O2").split()
    subprocess.run(["g++", *flags, "-std=c++17", "-ffp-contract=off", "-o", exe,
                    os.path.join(ROOT, "tests", "cpp", "og_driver.cpp"),
                    os.path.join(ROOT, "pacbio_amd", "csrc", "overlap_graph.cpp")], check=True)
    r = subprocess.run([exe, "graph", os.path.join(d, "params"), rf], capture_output=True, text=True,
                       env=dict(os.environ, OG_TIME="1"), check=True)
    with open(os.path.join(d, "out"), "w") as f:
        f.write(r.stdout)
    print(r.stderr.strip(), f"({n} reads)")


if __name__ == "__main__":
    main()
