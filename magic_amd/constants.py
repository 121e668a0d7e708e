"""``FLAGS`` / ``DISTANCE_METRICS`` mirror of ``11a/constants.py:5-91`` (only the fields the
training path reads). Values follow BASELINE.json: 100x100 shape pairs."""


class DISTANCE_METRICS:
    COSINE_DISTANCE = "Cosine distance"
    SQUARED_DIFFERENCE = "Squared difference"


class FLAGS:
    DATA_DIR = None                      # a directory or .zip of {N}_L.png / {N}_K.png pairs
    IMAGE_SIZE = 100                     # reference: 200 (11a/constants.py:32)
    NUM_EXAMPLES_TO_LOAD_INTO_QUEUE = 50
    NUM_EXAMPLES_PER_EPOCH_FOR_TRAIN = 960
    NUM_EXAMPLES_PER_EPOCH_FOR_EVAL = 400
    ROTATE = True
    NUM_LAYERS = 3 if ROTATE else 2
    BATCH_SIZE = 24
    DISTANCE_METRIC = DISTANCE_METRICS.SQUARED_DIFFERENCE
    USE_FP16 = False
    NUM_THREADS = 2
    RUN_INTERMEDIATE_TESTS = False
    PRINT_INFO = True


def metric_name(flag_value: str) -> str:
    if flag_value == DISTANCE_METRICS.COSINE_DISTANCE:
        return "cosine"
    if flag_value == DISTANCE_METRICS.SQUARED_DIFFERENCE:
        return "sqdiff"
    raise ValueError("Invalid distance metric: " + str(flag_value))
