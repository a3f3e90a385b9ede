"""Constants of parameters.rs (AlexandreGac/alphazero-chess @ 2025-08-24), runtime defaults here."""
ACTION_SPACE = 64 * 8 * 8          # parameters.rs:3
CACHE_CAPACITY = 500_000           # parameters.rs:4
SEED = 42                          # parameters.rs:6
NUM_RES_BLOCKS = 10                # parameters.rs:7
NUM_FILTERS = 128                  # parameters.rs:8
REPLAY_BUFFER_SIZE = 100_000       # parameters.rs:10
MIN_REPLAY_SIZE = 20_000           # parameters.rs:11
NUM_ITERATIONS = 10_000            # parameters.rs:12
NUM_EPISODES = 100                 # parameters.rs:13
NUM_THREADS = 8                    # parameters.rs:14
NUM_TRAIN_STEPS = 40               # parameters.rs:16
BATCH_SIZE = 512                   # parameters.rs:17
VALUE_LOSS_WEIGHT = 0.5            # parameters.rs:25
WEIGHT_DECAY = 1e-4                # parameters.rs:26
DIRICHLET_ALPHA = 0.3              # parameters.rs:28
DIRICHLET_EPSILON = 0.25           # parameters.rs:29
TEMPERATURE_ANNEALING = 15         # parameters.rs:31
NUM_SIMULATIONS = 256              # parameters.rs:32
TEMPERATURE = 1.0                  # parameters.rs:33 (only T = 1 is supported: visits^(1/T) = visits)
C_PUCT = 3.0                       # parameters.rs:34
EVALUATION_GAMES = 256             # parameters.rs:36
NUM_HALFMOVES = 100                # chess.rs:9
NUM_FULLMOVES = 200                # chess.rs:10
REPETITIONS = 3                    # chess.rs:11
