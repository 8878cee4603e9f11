"""The reference's training script (/root/reference/main.py) on this framework.

Same structure, call for call: U_net() (:36); an end-of-epoch LambdaCallback that
runs predict.py's conventions over images_to_predict/input (:39-69); paired
ImageDataGenerators with rescale 1/255, rotation 90, flips and zoom 0.2 over
data/train/{input1,output1} and data/test/{input1,output1}, seed 1, zipped
(:71-118); CSVLogger('log.csv', append=True, separator=';') (:121);
ModelCheckpoint("saved7-model-{epoch:02d}-{val_acc:.2f}.hdf5") (:123-124);
fit_generator(steps_per_epoch=1000, epochs=1000, validation_steps=100) (:126-132).

The only changes are the imports, the hyper-parameters exposed as flags (so a
smoke run can be short), and `dtype` (bf16 storage with fp32 accumulation
trains ~10x faster than fp32 on MI355X).  The augmenting generators run their
warps on the GPU and hand CUDA batches to fit_generator; checkpoints are Keras
HDF5 files.

    python examples/main.py --root <dir holding data/ and images_to_predict/> \\
        [--size 512] [--steps 1000] [--epochs 1000] [--val-steps 100] [--dtype bfloat16]
"""
import argparse
import glob
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cnn_itmo_amd import CSVLogger, LambdaCallback, ModelCheckpoint, U_net  # noqa: E402
from cnn_itmo_amd.datagen import ImageDataGenerator  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", default=".")
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--epochs", type=int, default=1000)
    ap.add_argument("--val-steps", type=int, default=100)
    ap.add_argument("--dtype", default="float32", choices=["float32", "bfloat16"])
    a = ap.parse_args(argv)
    os.chdir(a.root)
    S = a.size

    model = U_net(input_size=(S, S, 3), dtype=a.dtype)  # main.py:36

    def makePrediction(epoch, logs):  # main.py:39-67
        from PIL import Image
        os.makedirs("images_to_predict/output", exist_ok=True)
        for img in sorted(glob.glob("images_to_predict/input/*.png")):
            print("Grabbing ", 1, " input files")
            with Image.open(img) as openimg:
                X = np.asarray([np.true_divide(np.asarray(openimg.convert("RGB")).astype(float), 255)])
            pred = model.predict(X)
            imgpred = (pred * 255)[0].astype("uint8")
            Image.fromarray(imgpred).save("images_to_predict/output/" + "epochZZZ" + str(epoch)
                                          + os.path.basename(img))

    testmodelcb = LambdaCallback(on_epoch_end=makePrediction)  # main.py:69

    data_gen_args = dict(rescale=1. / 255, rotation_range=90, horizontal_flip=True, vertical_flip=True,
                         zoom_range=0.2)  # main.py:71-77
    image_datagen = ImageDataGenerator(**data_gen_args)
    mask_datagen = ImageDataGenerator(**data_gen_args)
    seed = 1
    flow = dict(target_size=(S, S), color_mode="rgb", class_mode=None, shuffle=True, seed=seed)
    image_generator = image_datagen.flow_from_directory("data/train/input1", batch_size=a.batch, **flow)
    mask_generator = mask_datagen.flow_from_directory("data/train/output1", batch_size=a.batch, **flow)
    train_generator = zip(image_generator, mask_generator)  # main.py:99
    testimage_generator = image_datagen.flow_from_directory("data/test/input1", batch_size=1, **flow)
    testmask_generator = mask_datagen.flow_from_directory("data/test/output1", batch_size=1, **flow)
    test_generator = zip(testimage_generator, testmask_generator)  # main.py:119

    csv_logger = CSVLogger("log.csv", append=True, separator=";")  # main.py:121
    filepath = "saved7-model-{epoch:02d}-{val_acc:.2f}.hdf5"
    checkpoint = ModelCheckpoint(filepath, verbose=1, save_best_only=False, mode="max")  # main.py:123-124

    return model.fit_generator(generator=train_generator, validation_data=test_generator,
                               validation_steps=a.val_steps, steps_per_epoch=a.steps, epochs=a.epochs, verbose=1,
                               callbacks=[csv_logger, checkpoint, testmodelcb])  # main.py:126-132


if __name__ == "__main__":
    main()
