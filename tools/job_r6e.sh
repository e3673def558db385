# round 6: where the fp8 streaming engine waits, two-phase vs one-phase step
set -o pipefail
for lib in build_f8trace build_f8onetrace vit.rs_amd_default build_f8one vit.rs_amd_default build_f8one; do
  L=vit.rs_amd/$lib/libvit_hip.so; [ "$lib" = vit.rs_amd_default ] && L=vit.rs_amd/libvit_hip.so
  echo "== $L"
  VIT_LIB=$L timeout -k 10 120 python3 tools/f8_trace.py --only fwd_qkv,dgrad_fc,fwd_fc,fwd_proj,dgrad_qkv,fwd_fcproj || exit 1
done
