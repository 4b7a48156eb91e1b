"""Synthetic stand-ins for the course datasets (SURVEY §2.1 H2, §2.8 "Datasets").

The reference copies its datasets from blob storage at runtime
(Includes/Classroom-Setup.py:38); there is no network here, so every dataset
is generated with the SAME schema, file layout and relative path, and with
planted structure where a notebook asserts on it (e.g. 103,000 people ->
100,000 after case/SSN-format-insensitive dedup, Labs/ML 00L:35-38; a MovieLens
ratings matrix of true rank 12 so the ALS CV picks rank 12, MLE 01:202; the
IoT table of ML 13:35-42 exactly as specified).

``install_datasets(root)`` writes::

    airbnb/sf-listings/sf-listings-2019-03-06.csv                 raw, "$1,234" prices
    airbnb/sf-listings/sf-listings-2019-03-06-clean.parquet/      4 partitions
    airbnb/sf-listings/sf-listings-2019-03-06-clean.delta/        same, versioned
    airbnb/sf-listings/sf-listings-2019-03-06-clean-100p.parquet/ 100 part files
    airbnb/sf-listings/airbnb-cleaned-mlflow.csv                  all-numeric + zipcode (ML 12:34,131)
    airbnb/sf-listings/models/sf-listings-2019-03-06/pipeline_model
    dataframes/people-with-dups.txt                               ':'-separated
    movielens/ratings.parquet/, movielens/movies.parquet/
    COVID/coronavirusdataset/Time.csv
"""
from __future__ import annotations

import datetime
import os
from typing import Optional

import numpy as np
import pandas as pd

NEIGHBOURHOODS = [
    "Bayview", "Bernal Heights", "Castro/Upper Market", "Chinatown", "Crocker Amazon", "Diamond Heights",
    "Downtown/Civic Center", "Excelsior", "Financial District", "Glen Park", "Golden Gate Park", "Haight Ashbury",
    "Inner Richmond", "Inner Sunset", "Lakeshore", "Marina", "Mission", "Nob Hill", "Noe Valley", "North Beach",
    "Ocean View", "Outer Mission", "Outer Richmond", "Outer Sunset", "Pacific Heights", "Parkside", "Potrero Hill",
    "Presidio", "Presidio Heights", "Russian Hill", "Seacliff", "South of Market", "Treasure Island/YBI",
    "Twin Peaks", "Visitacion Valley", "West of Twin Peaks", "Western Addition"]  # 37 > maxBins=32 (ML 06:110)
PROPERTY_TYPES = ["Apartment", "House", "Condominium", "Guest suite", "Townhouse", "Boutique hotel", "Loft",
                  "Hostel", "Serviced apartment", "Bed and breakfast", "Hotel", "Guesthouse", "Other"]
ROOM_TYPES = ["Entire home/apt", "Private room", "Shared room"]
BED_TYPES = ["Real Bed", "Futon", "Pull-out Sofa", "Airbed", "Couch"]
CANCELLATION = ["strict_14_with_grace_period", "moderate", "flexible", "super_strict_30", "super_strict_60"]
REVIEW_COLS = ["review_scores_rating", "review_scores_accuracy", "review_scores_cleanliness",
               "review_scores_checkin", "review_scores_communication", "review_scores_location",
               "review_scores_value"]
KEEP = ["host_is_superhost", "cancellation_policy", "instant_bookable", "host_total_listings_count",
        "neighbourhood_cleansed", "latitude", "longitude", "property_type", "room_type", "accommodates",
        "bathrooms", "bedrooms", "beds", "bed_type", "minimum_nights", "number_of_reviews"] + REVIEW_COLS + ["price"]
NA_COLS = ["bathrooms", "bedrooms", "beds"] + REVIEW_COLS  # 10 "_na" indicator columns (ML 01:214-234)


def airbnb_raw(n: int = 7146, seed: int = 0) -> pd.DataFrame:
    """Raw listings with the 24 kept columns + a few extras (ML 01:32-93)."""
    rng = np.random.default_rng(seed)
    hood = rng.choice(len(NEIGHBOURHOODS), n, p=_zipf(len(NEIGHBOURHOODS), rng))
    hood_base = rng.uniform(90, 260, len(NEIGHBOURHOODS))
    lat0 = 37.76 + rng.normal(0, 0.02, len(NEIGHBOURHOODS))
    lon0 = -122.44 + rng.normal(0, 0.025, len(NEIGHBOURHOODS))
    room = rng.choice(3, n, p=[0.6, 0.36, 0.04])
    prop = rng.choice(len(PROPERTY_TYPES), n, p=_zipf(len(PROPERTY_TYPES), rng, 1.3))
    acc = np.clip(rng.poisson(2.5, n) + 1, 1, 16).astype(int)
    bedrooms = np.clip(np.round(acc / 2 + rng.normal(0, 0.6, n)), 0, 10)
    beds = np.clip(np.round(bedrooms + rng.normal(0.3, 0.6, n)), 0, 16)
    baths = np.clip(np.round((1 + bedrooms / 3 + rng.normal(0, 0.3, n)) * 2) / 2, 0, 8)
    rating = np.clip(100 - rng.gamma(1.5, 3.0, n), 20, 100).round()
    subs = [np.clip(np.round(10 - rng.gamma(1.2, 0.4, n)), 2, 10) for _ in range(6)]
    nrev = rng.negative_binomial(1, 0.03, n)
    min_n = np.where(rng.uniform(size=n) < 0.7, rng.integers(1, 4, n), rng.choice([7, 30, 60, 90, 365, 1000], n))
    mult = np.array([1.0, 0.45, 0.3])[room]
    price = (hood_base[hood] * mult * (0.55 + 0.22 * acc) * (0.9 + rating / 500.0) *
             np.exp(rng.normal(0, 0.3, n))).round()
    price = np.clip(price, 0, 10000)
    price[rng.uniform(size=n) < 0.001] = 0.0  # a few $0 listings get filtered in ML 01
    df = pd.DataFrame({
        "id": np.arange(958, 958 + n),
        "host_is_superhost": np.where(rng.uniform(size=n) < 0.3, "t", "f"),
        "cancellation_policy": rng.choice(CANCELLATION, n, p=[0.5, 0.3, 0.17, 0.02, 0.01]),
        "instant_bookable": np.where(rng.uniform(size=n) < 0.4, "t", "f"),
        "host_total_listings_count": rng.negative_binomial(1, 0.2, n).astype(float) + 1,
        "neighbourhood_cleansed": np.array(NEIGHBOURHOODS, dtype=object)[hood],
        "latitude": lat0[hood] + rng.normal(0, 0.006, n),
        "longitude": lon0[hood] + rng.normal(0, 0.006, n),
        "property_type": np.array(PROPERTY_TYPES, dtype=object)[prop],
        "room_type": np.array(ROOM_TYPES, dtype=object)[room],
        "accommodates": acc,
        "bathrooms": baths,
        "bedrooms": bedrooms,
        "beds": beds,
        "bed_type": rng.choice(BED_TYPES, n, p=[0.95, 0.02, 0.015, 0.01, 0.005]),
        "minimum_nights": min_n.astype(int),
        "number_of_reviews": nrev.astype(int),
        "review_scores_rating": rating,
        "review_scores_accuracy": subs[0], "review_scores_cleanliness": subs[1],
        "review_scores_checkin": subs[2], "review_scores_communication": subs[3],
        "review_scores_location": subs[4], "review_scores_value": subs[5],
        "price": ["${:,.2f}".format(p) for p in price],
        "description": [f"Lovely place, \"cozy\" and bright\nin {NEIGHBOURHOODS[h]}" for h in hood],
    })
    for c in NA_COLS:
        miss = rng.uniform(size=n) < (0.18 if c.startswith("review") else 0.005)
        df.loc[miss, c] = np.nan
    return df


def airbnb_clean(raw: Optional[pd.DataFrame] = None, seed: int = 0) -> pd.DataFrame:
    """The output of ML 01 - Data Cleansing: price parsed, $0 and min-nights>365 rows
    dropped, ints as doubles, ``*_na`` indicators, median imputation."""
    raw = airbnb_raw(seed=seed) if raw is None else raw
    df = raw[KEEP].copy()
    df["price"] = df["price"].str.replace("$", "", regex=False).str.replace(",", "", regex=False).astype(float)
    df = df[(df.price > 0) & (df.minimum_nights <= 365)].reset_index(drop=True)
    for c in df.columns:
        if df[c].dtype.kind in "iu":
            df[c] = df[c].astype(float)
    for c in NA_COLS:
        df[c + "_na"] = df[c].isna().astype(float)
    for c in NA_COLS:
        df[c] = df[c].fillna(df[c].median())
    return df


def airbnb_mlflow_csv(clean: Optional[pd.DataFrame] = None) -> pd.DataFrame:
    """All-numeric table with categoricals as BIGINT codes (schema of ML 12:131)."""
    clean = airbnb_clean() if clean is None else clean
    cols = ["host_total_listings_count", "neighbourhood_cleansed", "latitude", "longitude", "property_type",
            "room_type", "accommodates", "bathrooms", "bedrooms", "beds", "bed_type", "minimum_nights",
            "number_of_reviews"] + REVIEW_COLS + ["price"]
    out = clean[cols].copy()
    for c in ("neighbourhood_cleansed", "property_type", "room_type", "bed_type"):
        out[c] = pd.Categorical(out[c]).codes.astype(np.int64)
    # SF zip codes (941xx) keyed by neighbourhood; ML 12:34 / Labs/ML 08L:34 drop it, ML 05:69 and
    # Labs/ML 12L:35 keep it as a feature (SURVEY §2.8 "zipcode dropped for some uses")
    out.insert(4, "zipcode", (94102.0 + (out["neighbourhood_cleansed"] * 7) % 32).astype(float))
    return out


def people_with_dups(n_unique: int = 100000, n_dups: int = 3000, seed: int = 0) -> pd.DataFrame:
    """Labs/ML 00L: duplicated records differ only by name case and SSN hyphenation."""
    rng = np.random.default_rng(seed)
    first = np.array(["Carol", "James", "Mary", "John", "Patricia", "Robert", "Linda", "Michael", "Barbara",
                      "William", "Elizabeth", "David", "Jennifer", "Richard", "Maria", "Joseph", "Susan", "Thomas"])
    last = np.array(["Smith", "Johnson", "Williams", "Brown", "Jones", "Garcia", "Miller", "Davis", "Rodriguez",
                     "Martinez", "Hernandez", "Lopez", "Gonzalez", "Wilson", "Anderson", "Thomas", "Taylor"])
    ssn_num = 100000000 + rng.choice(899999999, n_unique, replace=False)  # Floyd sampling, no 7 GB arange
    ssn = [f"{s // 1000000:03d}-{(s // 10000) % 100:02d}-{s % 10000:04d}" for s in ssn_num]
    gender = rng.choice(["F", "M"], n_unique)
    birth = [(datetime.date(1950, 1, 1) + datetime.timedelta(days=int(d))).isoformat() + "T05:00:00.000+0000"
             for d in rng.integers(0, 18000, n_unique)]
    df = pd.DataFrame({"firstName": rng.choice(first, n_unique), "middleName": rng.choice(first, n_unique),
                       "lastName": rng.choice(last, n_unique), "gender": gender, "birthDate": birth, "ssn": ssn,
                       "salary": rng.integers(20000, 200000, n_unique)})
    dup_idx = rng.choice(n_unique, n_dups, replace=False)
    d = df.iloc[dup_idx].copy()
    for c in ("firstName", "middleName", "lastName"):
        d[c] = d[c].str.upper()
    d["ssn"] = d["ssn"].str.replace("-", "", regex=False)
    out = pd.concat([df, d], ignore_index=True)
    return out.sample(frac=1.0, random_state=seed).reset_index(drop=True)


def movielens(n_users: int = 6040, n_movies: int = 3706, n_ratings: int = 1000000, rank: int = 12,
              seed: int = 0):
    """ratings(userId, movieId, rating) from a rank-12 factor model + movies(ID, title)."""
    rng = np.random.default_rng(seed)
    U = rng.normal(0, 1.0 / np.sqrt(rank), (n_users, rank))
    V = rng.normal(0, 1.0 / np.sqrt(rank), (n_movies, rank))
    bu = rng.normal(0, 0.3, n_users)
    bi = rng.normal(0, 0.4, n_movies)
    pop = _zipf(n_movies, rng, 0.8)
    u = rng.integers(0, n_users, n_ratings)
    i = rng.choice(n_movies, n_ratings, p=pop)
    key = u.astype(np.int64) * n_movies + i
    _, first = np.unique(key, return_index=True)
    u, i = u[first], i[first]
    r = 3.6 + bu[u] + bi[i] + 2.0 * (U[u] * V[i]).sum(1) + rng.normal(0, 0.3, len(u))
    ratings = pd.DataFrame({"userId": u + 1, "movieId": i + 1, "rating": np.clip(np.round(r), 1, 5)})
    movies = pd.DataFrame({"ID": np.arange(1, n_movies + 1), "title": [f"Movie {k} ({1950 + k % 70})"
                                                                      for k in range(1, n_movies + 1)]})
    return ratings, movies


def iot(spark, n: int = 1000 * 100):
    """ML 13:35-42 exactly: record_id, device_id = id % 10, feature_k = rand()*k, label."""
    from ..sql.functions import col, rand
    return (spark.range(n)
            .withColumn("device_id", (col("id") % 10).cast("int"))
            .withColumn("feature_1", rand() * 1)
            .withColumn("feature_2", rand() * 2)
            .withColumn("feature_3", rand() * 3)
            .withColumn("label", (col("feature_1") + col("feature_2") + col("feature_3")) + rand())
            .withColumnRenamed("id", "record_id"))


def covid_time(days: int = 163, seed: int = 0) -> pd.DataFrame:
    """COVID/coronavirusdataset/Time.csv: date,time,test,negative,confirmed,released,deceased."""
    rng = np.random.default_rng(seed)
    t = np.arange(days)
    confirmed = np.round(11000 / (1 + np.exp(-(t - 45) / 6.0)) + t * 8 + rng.normal(0, 20, days)).clip(1)
    confirmed = np.maximum.accumulate(confirmed).astype(int)
    released = np.maximum.accumulate(np.round(confirmed * np.clip((t - 30) / 80.0, 0, 0.92))).astype(int)
    deceased = np.maximum.accumulate(np.round(confirmed * 0.022 * np.clip(t / 60.0, 0, 1))).astype(int)
    test = np.maximum.accumulate(np.round(np.cumsum(200 + 9000 / (1 + np.exp(-(t - 40) / 5.0))))).astype(int)
    dates = [(datetime.date(2020, 1, 20) + datetime.timedelta(days=int(k))).isoformat() for k in t]
    return pd.DataFrame({"date": dates, "time": 16, "test": test, "negative": (test - confirmed) * 9 // 10,
                         "confirmed": confirmed, "released": released, "deceased": deceased})


def _zipf(k, rng, a=1.0):
    w = 1.0 / np.arange(1, k + 1) ** a
    w = w[rng.permutation(k)]
    return w / w.sum()


def install_datasets(root: str, spark=None, reinstall: bool = False, scale: float = 1.0) -> str:
    """Write every course dataset under ``root`` (H2 ``install_datasets``; skips existing
    files unless ``reinstall``).  ``scale`` shrinks row counts for fast tests."""
    from ..session import SparkSession
    spark = spark or SparkSession.builder.getOrCreate()
    marker = os.path.join(root, "_SUCCESS")
    if os.path.exists(marker) and not reinstall:
        return root
    os.makedirs(root, exist_ok=True)
    sf = os.path.join(root, "airbnb", "sf-listings")
    os.makedirs(sf, exist_ok=True)
    raw = airbnb_raw(n=max(200, int(7146 * scale)))
    raw.to_csv(os.path.join(sf, "sf-listings-2019-03-06.csv"), index=False)
    clean = airbnb_clean(raw)
    cdf = spark.createDataFrame(clean)
    cdf.repartition(4).write.mode("overwrite").parquet(os.path.join(sf, "sf-listings-2019-03-06-clean.parquet"))
    cdf.repartition(4).write.format("delta").mode("overwrite").save(
        os.path.join(sf, "sf-listings-2019-03-06-clean.delta"))
    cdf.repartition(100).write.mode("overwrite").parquet(
        os.path.join(sf, "sf-listings-2019-03-06-clean-100p.parquet"))
    airbnb_mlflow_csv(clean).to_csv(os.path.join(sf, "airbnb-cleaned-mlflow.csv"), index=False)
    # pre-trained pipeline model for MLE 00 (deployment / streaming)
    from ..ml import Pipeline
    from ..ml.feature import RFormula
    from ..ml.regression import RandomForestRegressor
    pm = Pipeline(stages=[RFormula(formula="price ~ .", featuresCol="features", labelCol="price",
                                   handleInvalid="skip"),
                          RandomForestRegressor(labelCol="price", maxBins=40, numTrees=10, maxDepth=5, seed=42)])
    pm.fit(cdf).write().overwrite().save(os.path.join(sf, "models", "sf-listings-2019-03-06", "pipeline_model"))
    ddir = os.path.join(root, "dataframes")
    os.makedirs(ddir, exist_ok=True)
    people = people_with_dups(n_unique=max(1000, int(100000 * scale)), n_dups=max(30, int(3000 * scale)))
    people.to_csv(os.path.join(ddir, "people-with-dups.txt"), sep=":", index=False)
    ml = os.path.join(root, "movielens")
    ratings, movies = movielens(n_users=max(300, int(6040 * scale)), n_movies=max(200, int(3706 * scale)),
                                n_ratings=max(20000, int(1000000 * scale)))
    spark.createDataFrame(ratings).write.mode("overwrite").parquet(os.path.join(ml, "ratings.parquet"))
    spark.createDataFrame(movies).write.mode("overwrite").parquet(os.path.join(ml, "movies.parquet"))
    cv = os.path.join(root, "COVID", "coronavirusdataset")
    os.makedirs(cv, exist_ok=True)
    covid_time().to_csv(os.path.join(cv, "Time.csv"), index=False)
    with open(marker, "w") as f:
        f.write(datetime.datetime.now().isoformat())
    return root
