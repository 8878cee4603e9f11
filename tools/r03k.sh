set -e
R=$GRAFT_REPO_ROOT
for v in rpf1 rpf2 rearly rpf1e; do
  bash tools/ab_layers.sh $R/cnn_itmo_amd/lib/variants/lib$v.so enc1b,dec9b,dec9,dec8,dec7,dec6 dgradbn
done
