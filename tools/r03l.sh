set -e
R=$GRAFT_REPO_ROOT
bash tools/ab_layers.sh $R/cnn_itmo_amd/lib/variants/libm32.so enc3b,enc4b,crossb,dec6,dec7,dec8,dec9b fwd,dgrad,dgradbn
