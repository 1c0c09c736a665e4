'''
Single-process MNIST CNN trainer -- the reference's mnist_single.py on the MI355X-native stack
(/root/reference/mnist_single.py:1-134).

Same constants (learning_rate 0.01, training_iters 4000, batch_size 128, display_step 10,
dropout 0.75), same model (conv5x5x32-pool-conv5x5x64-pool-fc1024-dropout-fc10, N(0,1) init),
same loop (`while step * batch_size < training_iters`, a keep_prob=1 minibatch-loss forward every
display_step), same 50 x 100 validation pass and the same stdout lines. On a GPU it runs the
native HIP engine (one captured hipGraph per step); without one, fp32 PyTorch on the CPU.
Optional overrides: --training_iters --batch_size --learning_rate --cpu --data_dir --seed.
'''
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from tensorflow_distributed_amd.models import mnist_cnn as M  # noqa: E402
from tensorflow_distributed_amd.models.mnist_runner import make_runner  # noqa: E402
from tensorflow_distributed_amd.training.optimizers import AdamOptimizer  # noqa: E402
from tensorflow_distributed_amd.utils import input_data  # noqa: E402

# Parameters (mnist_single.py:17-21)
learning_rate = 0.01
training_iters = 4000
batch_size = 128
display_step = 10

# Network Parameters (mnist_single.py:23-26)
n_input = 784  # MNIST data input (img shape: 28*28)
n_classes = 10  # MNIST total classes (0-9 digits)
dropout = 0.75  # Dropout, probability to keep units


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--training_iters", type=int, default=training_iters)
    ap.add_argument("--batch_size", type=int, default=batch_size)
    ap.add_argument("--learning_rate", type=float, default=learning_rate)
    ap.add_argument("--display_step", type=int, default=display_step)
    ap.add_argument("--data_dir", default="MNIST_data/")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu", action="store_true", help="force the fp32 PyTorch CPU path")
    ap.add_argument("--no_graph", action="store_true", help="GPU: launch kernels per step (no hipGraph)")
    ap.add_argument("--eval_batches", type=int, default=50)
    ap.add_argument("--train_flag", type=int, default=1, help="1 = train, else evaluation only (mnist_single.py:103)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"], help="GPU compute precision (fp32 = the "
                    "reference's)")
    ap.add_argument("--host_feed", action="store_true", help="GPU: feed every batch from the host (next_batch + "
                    "H2D) instead of the device-resident split with a per-epoch device shuffle")
    a = ap.parse_args(argv)

    # Import MNIST data (mnist_single.py:14-15)
    mnist = input_data.read_data_sets(a.data_dir, one_hot=True, seed=a.seed)
    dev = torch.device("cuda", 0) if (torch.cuda.is_available() and not a.cpu) else torch.device("cpu")
    runner = make_runner(a.batch_size, AdamOptimizer(a.learning_rate), dev, keep_prob=dropout, seed=a.seed,
                         use_graph=not a.no_graph, dtype=a.dtype)
    runner.load_flat(M.flat_from_dict(M.init_params(a.seed)), {}, 0)  # init = initialize_all_variables()
    device_input = dev.type == "cuda" and not a.host_feed
    if device_input:  # upload the split once; batches are gathered on the GPU (no per-step feed)
        runner.set_device_dataset(mnist.train.images, mnist.train.labels, seed=a.seed + 101)

    start_time = time.time()
    train_flag = a.train_flag
    step = 1
    if train_flag == 1:
        # Keep training until reach max iterations
        while step * a.batch_size < a.training_iters:
            if device_input:
                runner.train_step(None, None)  # next_batch happens on the device
            else:
                batch_x, batch_y = mnist.train.next_batch(a.batch_size)
                # Run optimization op (backprop)
                runner.train_step(batch_x, batch_y)
            if step % a.display_step == 0:
                if device_input:
                    batch_x, batch_y = runner.last_device_batch()
                # Calculate batch loss (keep_prob = 1)
                loss_sum, _ = runner.evaluate(batch_x, batch_y)
                loss = loss_sum / len(batch_x)
                print("Iter " + str(step * a.batch_size) + ", Minibatch Loss= " + "{:.6f}".format(loss))
            step += 1
        print("Optimization Finished!")
        training_end_time = time.time()
        print("--- %s seconds Time for Training ---" % (training_end_time - start_time))
    else:
        training_end_time = start_time
    # Calculate accuracy for 5000 mnist validation images
    nt = a.eval_batches
    accuracy_arr = []
    for counter in range(1, nt + 1):
        val_x, val_y = mnist.validation.next_batch(100)
        _, correct = runner.evaluate(val_x, val_y)
        accuracy_arr.append(correct / float(len(val_x)))
    mean_accuracy = sum(accuracy_arr) / len(accuracy_arr)
    print("Mean Accuracy : %f" % mean_accuracy)
    testing_end_time = time.time()
    print("--- %s seconds Time for Inference ---" % (testing_end_time - training_end_time))
    return 0


if __name__ == '__main__':
    sys.exit(main())
