# Round 5, call G: attack-window calibration sweep 3 (contrast spread, a one-row sky band) with
# two warm-start lengths each (robustness of the trajectory to the starting point).
export SETS="c_ct03|cifar_params.yaml|synthetic_contrast=[0.3,1.2]
c_ct03_p44|cifar_params.yaml|synthetic_contrast=[0.3,1.2] pretrain_rounds=44
c_ct02|cifar_params.yaml|synthetic_contrast=[0.2,1.4]
c_ct02_p44|cifar_params.yaml|synthetic_contrast=[0.2,1.4] pretrain_rounds=44
c_sky30r1|cifar_params.yaml|synthetic_sky=0.3 synthetic_sky_rows=1
c_sky30r1_p44|cifar_params.yaml|synthetic_sky=0.3 synthetic_sky_rows=1 pretrain_rounds=44
c_sky15r1|cifar_params.yaml|synthetic_sky=0.15 synthetic_sky_rows=1
c_sky15r1_p44|cifar_params.yaml|synthetic_sky=0.15 synthetic_sky_rows=1 pretrain_rounds=44
m_m4_s5_p44|mnist_params.yaml|synthetic_margin=4 synthetic_shared=0.5 pretrain_rounds=44"
OUT=r5g bash scripts/gpu/r5_e.sh
