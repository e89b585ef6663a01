# End-to-end: cli.py on the reference's pickle format with checkpointing, then a resumed run.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/e2e      # logs only (data and checkpoints stay in the box's /tmp)
W=$(mktemp -d /tmp/e2e.XXXX)
mkdir -p $O
python tools/make_pickles.py $W/data 1200 > $O/make.log 2>&1 && \
COMMON="model.architecture=neutron dataset.zdc_type=neutron dataset.input_image_shape=[44,44] model.n_experts=1 train.batch_size=128 dataset.source=pickle dataset.DATA_IMAGES_PATH=$W/data/images.pkl dataset.DATA_COND_PATH=$W/data/cond.pkl dataset.DATA_POSITIONS_PATH=$W/data/pos.pkl train.precision=bf16 train.save_experiment_data=True train.ws_threshold_model_save=1e9 config.experiment_dir=$W/exp train.save_experiments_dir=" && \
timeout -k 10 300 python cli.py --max-steps-per-epoch 3 -o $COMMON train.epochs=1 > $O/run1.log 2>&1 && \
ls $W/exp/models $W/exp/info > $O/files.log 2>&1 && \
timeout -k 10 300 python cli.py --max-steps-per-epoch 3 -o $COMMON train.epochs=2 train.checkpoint_experiment_dir=$W/exp train.epoch_to_load=0 > $O/run2.log 2>&1
