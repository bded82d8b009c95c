# same-box A/B of two library builds on the per-task protocol (tools only)
set -e
for rep in 1 2 3; do
for lib in libbcp_old.so libbcp.so; do
BCP_LIB=$PWD/beegfs-chunk-parity_amd/lib/$lib TMPDIR=/dev/shm timeout -k 10 200 python tools/exp/proto_noop.py --reps 9 --lanes 12 2>>gpurun_out/ab_proto.err | sed "s/^{/{\"lib\": \"$lib\", /" >> gpurun_out/ab_proto.jsonl
done; done
