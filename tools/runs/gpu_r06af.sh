#!/bin/bash
# r06af: determinism of the final tree's whole frames after the MIS-record fix -- 60 renders of
# C3 (1920x1080@1024), 40 of C2 (700x700@256) and 20 of C5 (600x600@512), each against its golden
OUT=$PWD/gpurun_out/r06af
mkdir -p $OUT
export TMPDIR=/tmp
for fr in "bunny_frame_c3_1920x1080s1024 60" "killeroo_frame_c2_700x700s256 40" "anim_frame_c5_600x600s512 20"; do
set -- $fr
timeout -k 10 600 python3 tools/frame_repeat.py $1 $2 > $OUT/$1.jsonl 2> $OUT/$1.err || { tail -5 $OUT/$1.err; exit 1; }
python3 -c "
import json;r=[json.loads(l) for l in open('$OUT/$1.jsonl')];print('$1', len(r), 'renders,', sum(1 for x in r if x['n_bad']), 'with tiles off the golden,', sum(1 for x in r if x['n_pix_diff']), 'differing from the first')"
done
echo done
