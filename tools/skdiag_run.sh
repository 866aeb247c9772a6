set -o pipefail
mkdir -p gpurun_out
for v in "" _noreduce _nopub; do
  MAECLIP_LIB=$PWD/mae_clip_amd/libmaeclip$v.so timeout -k 10 120 python -u tools/sk_diag.py "lib$v" >> gpurun_out/skdiag_r5c.jsonl 2>gpurun_out/skdiag_r5c.err || exit 1
done
STAMPS=1 MAECLIP_LIB=$PWD/mae_clip_amd/libmaeclip_stamps.so timeout -k 10 120 python -u tools/sk_diag.py "lib_stamps" >> gpurun_out/skdiag_r5c.jsonl 2>>gpurun_out/skdiag_r5c.err
