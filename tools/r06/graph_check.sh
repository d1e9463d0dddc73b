#!/bin/bash
# Round 6: the bounds-checking build of the graph kernels (-DPBGPU_GRAPH_CHECK,
# pacbio_amd/libpbgpu_gcheck.so) under bin/create_mega_reads (LD_LIBRARY_PATH puts it
# before the product library) on all 20k C4r and all 50k C2 reads, the run path's many
# batches on two aligners; prints the violation counters and compares the output with the
# product library's.  Usage: bash tools/r06/graph_check.sh OUTDIR
O=$1; mkdir -p $O/gck_lib
ln -sf "$GRAFT_REPO_ROOT/pacbio_amd/libpbgpu_gcheck.so" $O/gck_lib/libpbgpu.so
for wl in "C4r 20000" "C2 50000"; do
  W=${wl% *}; N=${wl#* }
  D=/tmp/gck_$W; mkdir -p $D
  python3 -c "import sys; sys.path.insert(0, '.'); from tools.synth import Dataset; d = Dataset('$W', seed=42, threads=16, n_pb=$N); d.write('$D')" || exit 1
  F="-s 1M -m 17 --psa-min 13 -k 31 -l $D/ul.txt -B 15 --max-count 5000 --stretch-cap 10000 -t 16 --timing -r $D/sr.fa -p $D/pb.fa"
  timeout -k 10 300 pacbio_amd/bin/create_mega_reads $F -o $D/prod.txt 2> $O/gck_${W}_prod.err || exit $?
  LD_LIBRARY_PATH=$GRAFT_REPO_ROOT/$O/gck_lib timeout -k 10 300 pacbio_amd/bin/create_mega_reads $F -o $D/chk.txt 2> $O/gck_${W}_chk.err || exit $?
  echo "$W: $(grep 'graph-check' $O/gck_${W}_chk.err) output $(cmp -s $D/prod.txt $D/chk.txt && echo identical || echo DIFFERS) ($(wc -c < $D/prod.txt) bytes)" >> $O/graph_check.txt
  rm -rf $D
done
cat $O/graph_check.txt
