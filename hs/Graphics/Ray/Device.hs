{-# LANGUAGE DataKinds #-}
{-# LANGUAGE DeriveFunctor #-}
{-# LANGUAGE ForeignFunctionInterface #-}
{-# LANGUAGE PatternSynonyms #-}
{-# LANGUAGE RecordWildCards #-}
{-# LANGUAGE ScopedTypeVariables #-}
{-# LANGUAGE ViewPatterns #-}
-- | MI355X drop-in for 'Graphics.Ray.raytrace' (reference: src/Graphics/Ray.hs:121-238).
--
-- Switch a program from the CPU ray tracer to the GPU by importing this module instead of
-- "Graphics.Ray": it exports the same names with the same arguments —
--
-- > raytrace :: ToRandom m => CameraSettings -> Geometry m Material -> StdGen -> A.Matrix D Color
--
-- and the smart constructors of Geometry.hs:5-16, Material.hs:3-6 and Texture.hs:2-5
-- ('sphere', 'parallelogram', 'group', 'bvhTree', 'transform', 'moving', 'constantMedium',
-- 'lambertian', 'dielectric', 'checkerTexture', ...).  The reference's geometries, materials
-- and textures are closures (Geometry.hs:42, Material.hs:17, Texture.hs:15), which the device
-- cannot evaluate, so every value built here carries BOTH the reference closure (built by the
-- reference's own constructor) and a description of what it is.  The reference's raw
-- constructors are exported under the same names ('Geometry', 'Material', 'Texture': bundled
-- pattern synonyms with the reference's fields), so user-defined geometries, materials and
-- textures compile unchanged; they carry no description and render through the CPU fallback
-- ('fromReferenceGeometry', 'fromReferenceMaterial' and 'fromReferenceTexture' lift existing
-- reference values the same way).  'raytrace' flattens the
-- description into the records of include/rt.h and calls rt_render (binary64, every visible
-- GPU); when any part of the scene is an arbitrary closure ('solidTexture', 'uvTexture',
-- 'planeShape' with a user predicate, a background that is not @const c@ or a y-lerp, a
-- non-Euclidean 'transform') or the library reports RT_E_UNSUPPORTED, it evaluates the
-- reference closure with the reference's CPU 'Graphics.Ray.raytrace' instead.  Either way the
-- result is the h x w matrix of linear colours (row 0 at the top) of Ray.hs:238.
--
-- SOURCE ONLY: GHC is not available in the build container, so this module is not compiled or
-- tested here.  The C ABI it binds (include/rt.h) is exercised from Python (ctypes) and C by
-- tests/, the struct offsets below are checked against the C layout by
-- tests/test_abi.py::test_haskell_binding_offsets_match_header, and the flattening rules are the
-- ones raytrace_amd/scene.py implements and tests/ check against the oracle (INTEGRATION.md).
module Graphics.Ray.Device
  ( -- * The drop-in
    raytrace, raytraceWith, DeviceOptions(..), defaultDeviceOptions, Precision(..), RenderError(..)
  , renderOnDevice, deviceCount
    -- * 8-bit output encoded on the device (writeImage / writeImageSqrt of a render, Ray.hs:248-260)
  , Encoding(..), renderImage8, raytraceToFile
    -- * Geometry (Geometry.hs:5-16)
  , Geometry(Geometry), boundingBox, pureGeometry, transform, moving
  , sphere, planeShape, parallelogram, cuboid, triangle, triangleMesh, constantMedium
  , group, bvhNode, bvhTree
    -- * Materials (Material.hs:3-6)
  , Material(Material), R.MaterialResult(..)
  , lightSource, pitchBlack, lambertian, lommelSeeliger, mirror, metal, dielectric, transparent
  , isotropic, anisotropic
    -- * Textures (Texture.hs:2-5)
  , Texture(Texture), constantTexture, solidTexture, uvTexture, imageTexture, checkerTexture, noiseTexture
  , marbleTexture
    -- * Between the reference's values and these
  , toReference, toReferenceRandom, referenceMaterial, referenceTexture
  , fromReferenceGeometry, fromReferenceMaterial, fromReferenceTexture
    -- * Unchanged from the reference
  , R.CameraSettings(..), R.defaultCameraSettings, R.ToRandom, R.Mesh(R.Mesh), R.transformVertices, R.parseObj
  , R.readObj, R.translate, R.rotateX, R.rotateY, R.rotateZ, R.scale, R.readImage, R.writeImage, R.writeImageSqrt
  , module Graphics.Ray.Core
  ) where

import qualified Graphics.Ray as R
import Graphics.Ray.Core

import Control.Monad (foldM, forM_, when, zipWithM_)
import Control.Monad.State (State, evalState)
import Data.Bits (shiftR, xor)
import Data.List (sortOn)
import Data.Functor.Identity (Identity)
import Data.Int (Int32)
import qualified Data.Map.Strict as Map
import Data.Word (Word64, Word8)
import qualified Data.Massiv.Array as A
import qualified Data.Massiv.Array.Unsafe as AU
import Foreign
import Foreign.C.String (CString, peekCString)
import Foreign.C.Types (CDouble, CFloat, CInt (..))
import Graphics.Pixel.ColorSpace (Linearity (NonLinear), SRGB)
import qualified Graphics.Pixel.ColorSpace as C
import qualified Data.Massiv.Array.IO as I
import Data.IORef (modifyIORef', newIORef, readIORef, writeIORef)
import System.Mem.StableName (StableName, eqStableName, hashStableName, makeStableName)
import Linear (M44, V2 (V2), V3 (V3), V4 (V4), cross, dot, norm, (!*))
import System.IO.Unsafe (unsafePerformIO)
import System.Random (StdGen, mkStdGen)
import System.Random.Internal (StdGen (unStdGen))
import System.Random.SplitMix (unseedSMGen)

-- ===================================================================== descriptions

-- | What a texture is, when it is one of the reifiable constructors (Texture.hs:18-78).
data TexD
  = TConst Color
  | TChecker Int Int Color Color
  | TImage Int Int Double [Color]                  -- ^ width, height, fingerprint, row-major texels (row 0 = top)
  | TNoise Int Double (V3 Double) Color Color     -- ^ layers, frequency, shift, colour 0, colour 1
  | TMarble Vec3 Double (V3 Double)                -- ^ stripe direction, frequency, shift

-- | The identity of a texture in the flattened tables (materials and textures are shared by
-- every leaf that uses them; an image is keyed by its size and a position-weighted checksum of
-- its texels, computed once per imageTexture).
data TexKey
  = KConst Color | KChecker Int Int Color Color | KImage Int Int Double
  | KNoise Int Double (V3 Double) Color Color | KMarble Vec3 Double (V3 Double)
  deriving (Eq, Ord)

texKey :: TexD -> TexKey
texKey t = case t of
  TConst c -> KConst c
  TChecker a b c d -> KChecker a b c d
  TImage w h f _ -> KImage w h f
  TNoise a b c d e -> KNoise a b c d e
  TMarble a b c -> KMarble a b c

-- | A material (Material.hs:41-129): the reference closure and, when its texture is reifiable,
-- its kind (rt.h RT_MAT_*), texture and parameter.
data Material = DeviceMaterial
  { matDesc :: Maybe (Int32, TexD, Double)
  , matRef :: R.Material
  }

-- | A texture: the reference closure and, for the reifiable constructors, its description.
data Texture = DeviceTexture
  { texDesc :: Maybe TexD
  , texRef :: R.Texture
  }

-- | The geometry tree as written (Geometry.hs:5-16): `group`, `bvhNode` and `bvhTree` are all
-- closest-hit groups (their result does not depend on the tree's shape, only on the
-- depth-first order of the leaves), `<$` is 'fmap'.  'DPlaced' is a `transform` tagged with the
-- identity of its child value (tagShared), so that placements of one shared object can share
-- one object-space BVH on the device.
data Desc a
  = DSphere Point3 Double a
  | DPlane Int32 Point3 Vec3 Vec3 (V2 Double) (V2 Double) (V2 Double) a  -- ^ rt.h kind 1 / 2
  | DGroup [Desc a]
  | DTransform (M44 Double) (Desc a)
  | DPlaced Int (M44 Double) (Desc a)
  | DMoving Vec3 Vec3 (Desc a)
  | DMedium Double (Desc ()) a
  deriving (Functor)

-- | A geometry: the reference value and, when every part is reifiable, its description.
data Geometry m a = DeviceGeometry
  { geoDesc :: Maybe (Desc a)
  , geoRef :: R.Geometry m a
  }

instance Functor m => Functor (Geometry m) where
  fmap f (DeviceGeometry d g) = DeviceGeometry (fmap (fmap f) d) (fmap f g)

-- | The reference's raw constructor (Geometry.hs:42): a user-defined geometry, rendered on the
-- CPU (its hit function is a closure).  Matching on it yields the reference value's fields.
pattern Geometry :: Box -> (Double -> Ray -> Interval -> m (Maybe (HitRecord, a))) -> Geometry m a
pattern Geometry box hit <- (geoRef -> R.Geometry box hit)
  where Geometry box hit = fromReferenceGeometry (R.Geometry box hit)
{-# COMPLETE Geometry #-}

-- | The reference's raw constructor (Material.hs:17): a user-defined material (README.md:11),
-- rendered on the CPU.
pattern Material :: (Vec3 -> HitRecord -> (Color, State StdGen R.MaterialResult)) -> Material
pattern Material f <- (matRef -> R.Material f)
  where Material f = fromReferenceMaterial (R.Material f)
{-# COMPLETE Material #-}

-- | The reference's raw constructor (Texture.hs:15): a user-defined texture, rendered on the CPU.
pattern Texture :: (Point3 -> V2 Double -> Color) -> Texture
pattern Texture f <- (texRef -> R.Texture f)
  where Texture f = fromReferenceTexture (R.Texture f)
{-# COMPLETE Texture #-}

-- | Lift a reference value: no description, so a scene that contains it renders on the CPU
-- through the reference's own 'R.raytrace' — by construction, whatever the closure does.
fromReferenceGeometry :: R.Geometry m a -> Geometry m a
fromReferenceGeometry = DeviceGeometry Nothing

fromReferenceMaterial :: R.Material -> Material
fromReferenceMaterial = DeviceMaterial Nothing

fromReferenceTexture :: R.Texture -> Texture
fromReferenceTexture = DeviceTexture Nothing

-- | The reference geometry with the reference materials (what 'R.raytrace' takes).
toReference :: Functor m => Geometry m Material -> R.Geometry m R.Material
toReference = fmap matRef . geoRef

-- | The same, with its hit function lifted into 'State StdGen' by the reference's own
-- 'R.toRandom' — exactly what 'R.raytrace' applies to every hit (Ray.hs:178; for
-- @State StdGen@ its 'R.toRandom' is 'id'), so @R.raytrace cs (toReferenceRandom w)@ draws the
-- same numbers as @R.raytrace cs (toReference w)@ and the CPU fallback needs no constraint beyond
-- the reference's own @ToRandom m@ (Ray.hs:121).
toReferenceRandom :: R.ToRandom m => Geometry m Material -> R.Geometry (State StdGen) R.Material
toReferenceRandom g = case geoRef g of
  R.Geometry box hit -> R.Geometry box (\t r i -> fmap (fmap (fmap matRef)) (R.toRandom (hit t r i)))

referenceMaterial :: Material -> R.Material
referenceMaterial = matRef

referenceTexture :: Texture -> R.Texture
referenceTexture = texRef

-- ---------------------------------------------------------------- geometry constructors

boundingBox :: Geometry m a -> Box
boundingBox = R.boundingBox . geoRef

pureGeometry :: Applicative m => Geometry Identity a -> Geometry m a
pureGeometry (DeviceGeometry d g) = DeviceGeometry d (R.pureGeometry g)

sphere :: Point3 -> Double -> Geometry Identity ()
sphere c r = DeviceGeometry (Just (DSphere c r ())) (R.sphere c r)

-- | A plane shape with a caller predicate is an arbitrary closure: CPU only.
planeShape :: Point3 -> Vec3 -> Vec3 -> (Double -> Double -> Bool) -> (Double -> Double -> V2 Double) -> Box
           -> Geometry Identity ()
planeShape q u v test uv bbox = DeviceGeometry Nothing (R.planeShape q u v test uv bbox)

parallelogram :: Point3 -> Vec3 -> Vec3 -> Geometry Identity ()
parallelogram q u v =
  DeviceGeometry (Just (DPlane 1 q u v (V2 0 0) (V2 1 0) (V2 0 1) ())) (R.parallelogram q u v)

triangle :: (Point3, V2 Double) -> (Point3, V2 Double) -> (Point3, V2 Double) -> Geometry Identity ()
triangle a@(p0, uv0) b@(p1, uv1) c@(p2, uv2) =
  DeviceGeometry (Just (DPlane 2 p0 (p1 - p0) (p2 - p0) uv0 uv1 uv2 ())) (R.triangle a b c)

-- | Geometry.hs:154-166: six parallelograms in the reference's order.
cuboid :: Box -> Geometry Identity ()
cuboid box@(V3 (xmin, xmax) (ymin, ymax) (zmin, zmax)) =
  let dx = V3 (xmax - xmin) 0 0
      dy = V3 0 (ymax - ymin) 0
      dz = V3 0 0 (zmax - zmin)
      faces = [ parallelogram (V3 xmin ymin zmax) dx dy, parallelogram (V3 xmax ymin zmin) (-dx) dy
              , parallelogram (V3 xmin ymin zmin) dz dy, parallelogram (V3 xmax ymin zmax) (-dz) dy
              , parallelogram (V3 xmin ymax zmax) dx (-dz), parallelogram (V3 xmin ymin zmin) dx dz ]
  in DeviceGeometry (DGroup <$> traverse geoDesc faces) (R.cuboid box)

-- | Geometry.hs:288-294: the mesh's triangles with the reference's default texture coordinates.
triangleMesh :: R.Mesh -> Geometry Identity ()
triangleMesh mesh@(R.Mesh verts uvs tris) =
  let tri (V3 (i0, j0) (i1, j1) (i2, j2)) =
        let uv j d = maybe d (A.index' uvs) j
        in triangle (A.index' verts i0, uv j0 (V2 0 0)) (A.index' verts i1, uv j1 (V2 1 0))
                    (A.index' verts i2, uv j2 (V2 0 1))
  in DeviceGeometry (DGroup <$> traverse (geoDesc . tri) tris) (R.triangleMesh mesh)

constantMedium :: Double -> Geometry Identity () -> Geometry (State StdGen) ()
constantMedium density g = DeviceGeometry ((\d -> DMedium density d ()) <$> geoDesc g) (R.constantMedium density (geoRef g))

group :: Monad m => [Geometry m a] -> Geometry m a
group gs = DeviceGeometry (DGroup <$> traverse geoDesc gs) (R.group (map geoRef gs))

bvhNode :: Monad m => Geometry m a -> Geometry m a -> Geometry m a
bvhNode a b = DeviceGeometry (DGroup <$> traverse geoDesc [a, b]) (R.bvhNode (geoRef a) (geoRef b))

-- | The device builds its own BVH; the closest hit (and so the image) does not depend on it.
bvhTree :: Monad m => [Geometry m a] -> Geometry m a
bvhTree gs = DeviceGeometry (DGroup <$> traverse geoDesc gs) (R.bvhTree (map geoRef gs))

transform :: Functor m => M44 Double -> Geometry m a -> Geometry m a
transform m g = DeviceGeometry (DTransform m <$> geoDesc g) (R.transform m (geoRef g))

moving :: Functor m => Vec3 -> Vec3 -> Geometry m a -> Geometry m a
moving v0 v1 g = DeviceGeometry (DMoving v0 v1 <$> geoDesc g) (R.moving v0 v1 (geoRef g))

-- ---------------------------------------------------------------- materials and textures

mat :: Int32 -> Texture -> Double -> R.Material -> Material
mat k t p = DeviceMaterial ((\d -> (k, d, p)) <$> texDesc t)

lightSource, lambertian, lommelSeeliger, mirror, transparent, isotropic :: Texture -> Material
lightSource t = mat 0 t 0 (R.lightSource (texRef t))
lambertian t = mat 2 t 0 (R.lambertian (texRef t))
lommelSeeliger t = mat 3 t 0 (R.lommelSeeliger (texRef t))
mirror t = mat 4 t 0 (R.mirror (texRef t))
transparent t = mat 7 t 0 (R.transparent (texRef t))
isotropic t = mat 8 t 0 (R.isotropic (texRef t))

pitchBlack :: Material
pitchBlack = DeviceMaterial (Just (1, TConst (V3 0 0 0), 0)) R.pitchBlack

metal :: Double -> Texture -> Material
metal fuzz t = mat 5 t fuzz (R.metal fuzz (texRef t))

dielectric :: Double -> Material
dielectric ior = DeviceMaterial (Just (6, TConst (V3 0 0 0), ior)) (R.dielectric ior)

anisotropic :: Double -> Texture -> Material
anisotropic g t = mat 9 t g (R.anisotropic g (texRef t))

constantTexture :: Color -> Texture
constantTexture c = DeviceTexture (Just (TConst c)) (R.constantTexture c)

solidTexture :: (Point3 -> Color) -> Texture
solidTexture f = DeviceTexture Nothing (R.solidTexture f)

uvTexture :: (V2 Double -> Color) -> Texture
uvTexture f = DeviceTexture Nothing (R.uvTexture f)

imageTexture :: A.Manifest r Color => A.Matrix r Color -> Texture
imageTexture img =
  let A.Sz (h A.:. w) = A.size img
      texels = A.toList img
      fingerprint = sum (zipWith (\k (V3 r g b) -> fromIntegral (k + 1) * (r + 3 * g + 7 * b)) [0 :: Int ..] texels)
  in DeviceTexture (Just (TImage w h fingerprint texels)) (R.imageTexture img)

checkerTexture :: Int -> Int -> Color -> Color -> Texture
checkerTexture nu nv c0 c1 = DeviceTexture (Just (TChecker nu nv c0 c1)) (R.checkerTexture nu nv c0 c1)

noiseTexture :: Int -> Double -> V3 Double -> Color -> Color -> Texture
noiseTexture k f s c0 c1 = DeviceTexture (Just (TNoise k f s c0 c1)) (R.noiseTexture k f s c0 c1)

marbleTexture :: Vec3 -> Double -> V3 Double -> Texture
marbleTexture d f s = DeviceTexture (Just (TMarble d f s)) (R.marbleTexture d f s)

-- ===================================================================== flattening
-- raytrace_amd/scene.py:flatten, restated: rigid transforms and motion baked into the leaves,
-- the material of a surface is the outermost `<$` above it, `constantMedium`s lifted to the top
-- level with their boundary leaves in set k + 1, each leaf's depth-first `order` kept for the
-- tie-break, and a geometric identity `gid` shared by identical baked leaves in every set.

data Prim = Prim
  { pKind :: Int32, pMat :: Int32, pSet :: Int32, pMotion :: Int32, pGid :: Int32, pOrder :: Int32
  , pUvFrame :: Int32, pP :: [Double], pUv :: [Double] }

data Flat = Flat
  { fPrims :: [Prim]                        -- reversed while building
  , fMedia :: [(Double, Int32, Int32)]      -- (density, material, order), reversed
  , fMats :: Map.Map (Int32, Double, Int32) Int32   -- (kind, parameter, texture index) -> material index
  , fMatList :: [(Int32, Int32, Double)]    -- (kind, texture, param), reversed
  , fTexIx :: Map.Map TexKey Int32
  , fTexs :: [TexD]                         -- reversed
  , fMotions :: [(Vec3, Vec3)]              -- reversed
  , fFrames :: Map.Map [Double] Int32
  , fGids :: Map.Map (Int32, [Double], Maybe (Vec3, Vec3), Int32) Int32
  , fOrder :: Int32
  , fBlas :: Map.Map Int (Int32, Int32)     -- shared object (tagShared key) -> (object index, leaves)
  , fInstances :: [(Int32, Int32, M34)]     -- (object, depth-first order of its first leaf, placement), reversed
  }

-- | rt.h RT_SET_BLAS: the set of an instanced object's object-space leaves.
setBlas :: Int32 -> Int32
setBlas b = -1 - b

-- | A rigid `transform` over at least this many leaves is a two-level instance (rt_instance), not
-- baked (raytrace_amd/scene.py INSTANCE_MIN_LEAVES; smaller objects are cheaper to trace baked).
instanceMinLeaves :: Int
instanceMinLeaves = 64

leafCount :: Desc a -> Int
leafCount d = case d of
  DSphere{} -> 1
  DPlane{} -> 1
  DGroup cs -> sum (map leafCount cs)
  DTransform _ c -> leafCount c
  DPlaced _ _ c -> leafCount c
  DMoving _ _ c -> leafCount c
  DMedium _ b _ -> leafCount b

-- | Subtrees with `moving` or media stay baked (an instance has one rigid placement).
bakesOnly :: Desc a -> Bool
bakesOnly d = case d of
  DMoving{} -> True
  DMedium{} -> True
  DGroup cs -> any bakesOnly cs
  DTransform _ c -> bakesOnly c
  DPlaced _ _ c -> bakesOnly c
  _ -> False

-- | Tag every `transform`'s child with the identity of its VALUE (a StableName): the placements
-- of one shared object, e.g. @map (\m -> transform m bunny) placements@, get the same key and
-- share one object-space BVH (rt_instance), as raytrace_amd/scene.py does with object identity.
-- Children that are equal but separately built get separate keys: correct, only less shared.
tagShared :: forall a. Desc a -> IO (Desc a)
tagShared root = do
  table <- newIORef (Map.empty :: Map.Map Int [(StableName (Desc a), Int)])
  next <- newIORef (0 :: Int)
  let keyOf :: Desc a -> IO Int
      keyOf c = do
        sn <- makeStableName $! c
        bucket <- Map.findWithDefault [] (hashStableName sn) <$> readIORef table
        case [ k | (o, k) <- bucket, eqStableName o sn ] of
          (k : _) -> pure k
          [] -> do
            k <- readIORef next
            writeIORef next (k + 1)
            modifyIORef' table (Map.insert (hashStableName sn) ((sn, k) : bucket))
            pure k
      go :: Desc a -> IO (Desc a)
      go d = case d of
        DGroup cs -> DGroup <$> mapM go cs
        DTransform m c -> do
          k <- keyOf c
          DPlaced k m <$> go c
        DMoving v0 v1 c -> DMoving v0 v1 <$> go c
        _ -> pure d  -- leaves; a medium's boundary is always baked (its set is not 0)
  go root

-- | 3 x 4 affine part of a 4 x 4 matrix, row-major.
type M34 = [[Double]]

m34Of :: M44 Double -> M34
m34Of (V4 (V4 a b c d) (V4 e f g h) (V4 i j k l) _) = [[a, b, c, d], [e, f, g, h], [i, j, k, l]]

compose :: M34 -> M34 -> M34
compose o i =
  [ [ sum [ (o !! r !! k) * (i !! k !! c) | k <- [0 .. 2] ] + (if c == 3 then o !! r !! 3 else 0) | c <- [0 .. 3] ]
  | r <- [0 .. 2] ]

mulPoint, mulVector :: M34 -> V3 Double -> V3 Double
mulPoint m (V3 x y z) = let row r = (m !! r !! 0) * x + (m !! r !! 1) * y + (m !! r !! 2) * z + (m !! r !! 3) in V3 (row 0) (row 1) (row 2)
mulVector m (V3 x y z) = let row r = (m !! r !! 0) * x + (m !! r !! 1) * y + (m !! r !! 2) * z in V3 (row 0) (row 1) (row 2)

det3 :: M34 -> Double
det3 m = let e r c = m !! r !! c
  in e 0 0 * (e 1 1 * e 2 2 - e 1 2 * e 2 1) - e 0 1 * (e 1 0 * e 2 2 - e 1 2 * e 2 0) + e 0 2 * (e 1 0 * e 2 1 - e 1 1 * e 2 0)

-- | R^T R = I within 1e-9 (the reference documents Euclidean transforms only, Geometry.hs:379-381)
rigid :: M34 -> Bool
rigid m = and [ abs (sum [ (m !! k !! a) * (m !! k !! b) | k <- [0 .. 2] ] - (if a == b then 1 else 0)) <= 1e-9
              | a <- [0 .. 2], b <- [0 .. 2] ]

v3l :: V3 Double -> [Double]
v3l (V3 x y z) = [x, y, z]

v2l :: V2 Double -> [Double]
v2l (V2 x y) = [x, y]

-- | Flatten a reifiable scene; Nothing when a part is not reifiable (CPU fallback).
flatten :: Desc Material -> Maybe Flat
flatten root = execStateM (walk root Nothing Nothing 0) empty
  where
    empty = Flat [] [] Map.empty [] Map.empty [] [] Map.empty Map.empty 0 Map.empty []
    execStateM m s = case m s of
      Nothing -> Nothing
      Just ((), s') -> Just s'

-- A tiny state-and-failure monad, written out so the module needs no transformer beyond mtl's State.
type FM a = Flat -> Maybe (a, Flat)

-- The material of a surface leaf is its own payload: `mat <$ g` is fmap, so the outermost `<$`
-- has already replaced every payload below it (Geometry.hs:44-47).
walk :: Desc Material -> Maybe M34 -> Maybe (Vec3, Vec3) -> Int32 -> FM ()
walk node m34 mv set = case node of
  DGroup cs -> seqAll [ walk c m34 mv set | c <- cs ]
  DTransform m c ->
    let m3 = m34Of m
    in if not (rigid m3) then const Nothing
       else walk c (Just (maybe m3 (`compose` m3) m34)) mv set
  DPlaced key m c ->
    let m3 = m34Of m
        m2 = maybe m3 (`compose` m3) m34
    in if not (rigid m3) then const Nothing
       else if set /= 0 || mv /= Nothing || leafCount c < instanceMinLeaves || bakesOnly c
         then walk c (Just m2) mv set
         else \s0 -> do
           -- two-level instancing (rt_instance): the object's leaves once, in object space, in set
           -- RT_SET_BLAS(b) with orders 0 .. n-1; each placement takes the next n orders
           (b, n, s1) <- case Map.lookup key (fBlas s0) of
             Just (b, n) -> Just (b, n, s0)
             Nothing -> do
               let b = fromIntegral (Map.size (fBlas s0))
               ((), sObj) <- walk c Nothing Nothing (setBlas b) s0 { fOrder = 0 }
               let n = fOrder sObj
               Just (b, n, sObj { fOrder = fOrder s0, fBlas = Map.insert key (b, n) (fBlas sObj) })
           Just ((), s1 { fInstances = (b, fOrder s1, m2) : fInstances s1, fOrder = fOrder s1 + n })
  DMoving v0 v1 c ->
    let rot v = maybe v (`mulVector` v) m34
        (w0, w1) = (rot v0, rot v1)
        mv' = case mv of
          Nothing -> (w0, w1)
          Just (a0, a1) -> (w0 + a0, w1 + a1)
    in walk c m34 (Just mv') set
  DMedium dens boundary m -> \s ->
    if set /= 0 then Nothing else do
      (mi, s1) <- materialIndex m s
      let k = fromIntegral (length (fMedia s1)) :: Int32
          s2 = s1 { fMedia = (dens, mi, fOrder s1) : fMedia s1, fOrder = fOrder s1 + 1 }
      walk (fmap (const m) boundary) m34 mv (k + 1) s2
  DSphere c r m -> leaf m $ \s -> do
    let c' = maybe c (`mulPoint` c) m34
    (uvf, s1) <- frame s
    pure ((0, v3l c' ++ [r, 0, 0, 0, 0, 0], replicate 6 0, uvf), s1)
  DPlane kind q u v uv0 uv1 uv2 m -> leaf m $ \s -> do
    let (q', u0, v0) = case m34 of
          Nothing -> (q, u, v)
          Just t -> (mulPoint t q, mulVector t u, mulVector t v)
        reflected = maybe False ((< 0) . det3) m34
        (a0, a1, a2) = if kind == 1 then (V2 0 0, V2 1 0, V2 0 1) else (uv0, uv1, uv2)
        -- keep the reference's object-space front side under a reflection (swap u and v)
        (u', v', t1, t2) = if reflected then (v0, u0, a2, a1) else (u0, v0, a1, a2)
    pure ((kind, v3l q' ++ v3l u' ++ v3l v', v2l a0 ++ v2l t1 ++ v2l t2, -1), s)
  where
    frame s = case m34 of
      Nothing -> Just (-1, s)
      Just t ->
        let rt = [ t !! c !! r | r <- [0 .. 2], c <- [0 .. 2] ]  -- R^T, row-major (sphereUV in object space)
        in case Map.lookup rt (fFrames s) of
             Just i -> Just (i, s)
             Nothing -> let i = fromIntegral (Map.size (fFrames s)) in Just (i, s { fFrames = Map.insert rt i (fFrames s) })
    leaf m body s0 = do
      (mi, s1) <- if set <= 0 then materialIndex m s0 else Just (-1, s0)
      ((kind, p, uv, uvf), s2) <- body s1
      let (mo, s3) = case mv of
            Nothing -> (-1, s2)
            Just pair -> (fromIntegral (length (fMotions s2)), s2 { fMotions = pair : fMotions s2 })
          key = (kind, p, mv, min 0 set)  -- an instanced object's leaves: a gid space of their own
          (gid, s4) = case Map.lookup key (fGids s3) of
            Just g -> (g, s3)
            Nothing -> let g = fromIntegral (Map.size (fGids s3)) in (g, s3 { fGids = Map.insert key g (fGids s3) })
          prim = Prim kind mi set mo gid (fOrder s4) uvf p uv
      pure ((), s4 { fPrims = prim : fPrims s4, fOrder = fOrder s4 + 1 })

seqAll :: [FM ()] -> FM ()
seqAll [] s = Just ((), s)
seqAll (f : fs) s = f s >>= \((), s') -> seqAll fs s'

-- | The table index of a material (and of its texture), shared by every leaf that uses the same
-- (kind, parameter, texture); Nothing for a closure texture.
materialIndex :: Material -> FM Int32
materialIndex (DeviceMaterial Nothing _) _ = Nothing
materialIndex (DeviceMaterial (Just (kind, tex, param)) _) s0 =
  let tk = texKey tex
      (ti, s1) = case Map.lookup tk (fTexIx s0) of
        Just i -> (i, s0)
        Nothing -> let i = fromIntegral (Map.size (fTexIx s0))
                   in (i, s0 { fTexIx = Map.insert tk i (fTexIx s0), fTexs = tex : fTexs s0 })
      mk = (kind, param, ti)
  in Just $ case Map.lookup mk (fMats s1) of
       Just i -> (i, s1)
       Nothing -> let i = fromIntegral (Map.size (fMats s1))
                  in (i, s1 { fMats = Map.insert mk i (fMats s1), fMatList = (kind, ti, param) : fMatList s1 })

-- ===================================================================== the C ABI (include/rt.h)

data RtScene
data RtCamera
data RtExec
data RtStats

foreign import ccall safe "rt_render"
  c_rt_render :: Ptr RtCamera -> Ptr RtScene -> Word64 -> Ptr RtExec -> Ptr () -> Ptr RtStats -> IO CInt
foreign import ccall unsafe "rt_last_error"
  c_rt_last_error :: IO CString
foreign import ccall unsafe "rt_image_height"
  c_rt_image_height :: Ptr RtCamera -> IO CInt
foreign import ccall safe "rt_device_count"
  c_rt_device_count :: IO CInt

-- Struct layouts of include/rt.h (x86-64).  tests/test_abi.py checks every `-- LAYOUT` line
-- against the C compiler's offsetof / sizeof.
-- LAYOUT rt_prim 152
-- LAYOUT rt_prim.p 32
-- LAYOUT rt_prim.uv 104
-- LAYOUT rt_medium 16
-- LAYOUT rt_material 16
-- LAYOUT rt_material.param 8
-- LAYOUT rt_texture 128
-- LAYOUT rt_texture.c0 16
-- LAYOUT rt_texture.c1 40
-- LAYOUT rt_texture.params 64
-- LAYOUT rt_perlin 9216
-- LAYOUT rt_perlin.grad 3072
-- LAYOUT rt_motion 48
-- LAYOUT rt_uvframe 72
-- LAYOUT rt_scene 136
-- LAYOUT rt_scene.prims 8
-- LAYOUT rt_scene.media 24
-- LAYOUT rt_scene.materials 40
-- LAYOUT rt_scene.textures 56
-- LAYOUT rt_scene.motions 72
-- LAYOUT rt_scene.uvframes 88
-- LAYOUT rt_scene.texels 104
-- LAYOUT rt_scene.perlin 112
-- LAYOUT rt_scene.n_instances 120
-- LAYOUT rt_scene.instances 128
-- LAYOUT rt_instance 112
-- LAYOUT rt_instance.m 16
-- LAYOUT rt_redirect_target 80
-- LAYOUT rt_camera_settings 184
-- LAYOUT rt_camera_settings.image_width 88
-- LAYOUT rt_camera_settings.background_c0 104
-- LAYOUT rt_camera_settings.background_c1 128
-- LAYOUT rt_camera_settings.defocus_angle 152
-- LAYOUT rt_camera_settings.n_redirect_targets 168
-- LAYOUT rt_camera_settings.redirect_targets 176
-- LAYOUT rt_exec 32
-- LAYOUT rt_exec.flags 16
-- LAYOUT rt_exec.n_devices 20
-- LAYOUT rt_exec.devices 24

pokeDoubles :: Ptr a -> Int -> [Double] -> IO ()
pokeDoubles p off xs = zipWithM_ (\k x -> pokeByteOff p (off + 8 * k) (realToFrac x :: CDouble)) [0 ..] xs

pokeI32 :: Ptr a -> Int -> Int32 -> IO ()
pokeI32 = pokeByteOff

-- | Marshal a flattened scene into an rt_scene (all arrays live for the continuation).
withFlatScene :: Flat -> (Ptr RtScene -> IO a) -> IO a
withFlatScene Flat{..} k =
  let prims = reverse fPrims
      media = reverse fMedia
      mats = reverse fMatList
      texs = reverse fTexs
      motions = reverse fMotions
      frames = map fst (sortOn snd (Map.toList fFrames))
      nTex = length texs
      images = [ cs | TImage _ _ _ cs <- texs ]
      texels = concat images
      needPerlin = or [ True | TNoise{} <- texs ] || or [ True | TMarble{} <- texs ]
      insts = reverse fInstances
  in allocaBytes (max 1 (152 * length prims)) $ \pp ->
     allocaBytes (max 1 (112 * length insts)) $ \pin ->
     allocaBytes (max 1 (16 * length media)) $ \pm ->
     allocaBytes (max 1 (16 * length mats)) $ \pmat ->
     allocaBytes (max 1 (128 * nTex)) $ \pt ->
     allocaBytes (max 1 (48 * length motions)) $ \pmo ->
     allocaBytes (max 1 (72 * length frames)) $ \pf ->
     allocaBytes (max 1 (12 * length texels)) $ \ptx ->
     allocaBytes 9216 $ \pper ->
     allocaBytes 136 $ \sc -> do
       fillBytes pp 0 (152 * length prims)
       forM_ (zip [0 ..] prims) $ \(i, Prim{..}) -> do
         let b = pp `plusPtr` (152 * i)
         pokeI32 b 0 pKind >> pokeI32 b 4 pMat >> pokeI32 b 8 pSet >> pokeI32 b 12 pMotion
         pokeI32 b 16 pGid >> pokeI32 b 20 pOrder >> pokeI32 b 24 pUvFrame >> pokeI32 b 28 0
         pokeDoubles b 32 pP >> pokeDoubles b 104 pUv
       forM_ (zip [0 ..] media) $ \(i, (d, m, o)) -> do
         let b = pm `plusPtr` (16 * i)
         pokeDoubles b 0 [d] >> pokeI32 b 8 m >> pokeI32 b 12 o
       forM_ (zip [0 ..] mats) $ \(i, (kind, t, p)) -> do
         let b = pmat `plusPtr` (16 * i)
         pokeI32 b 0 kind >> pokeI32 b 4 t >> pokeDoubles b 8 [p]
       fillBytes pt 0 (128 * nTex)
       let imageStarts = scanl (+) 0 [ w * h | TImage w h _ _ <- texs ]
       _ <- foldM (\imgNo (i, t) -> do
         let b = pt `plusPtr` (128 * i)
         pokeI32 b 12 (-1)
         case t of
           TConst c -> pokeI32 b 0 0 >> pokeDoubles b 16 (v3l c) >> pure imgNo
           TChecker nu nv c0 c1 -> do
             pokeI32 b 0 1 >> pokeI32 b 4 (fromIntegral nu) >> pokeI32 b 8 (fromIntegral nv)
             pokeDoubles b 16 (v3l c0) >> pokeDoubles b 40 (v3l c1) >> pure imgNo
           TImage w h _ _ -> do
             pokeI32 b 0 2 >> pokeI32 b 4 (fromIntegral w) >> pokeI32 b 8 (fromIntegral h)
             pokeI32 b 12 (fromIntegral (imageStarts !! imgNo)) >> pure (imgNo + 1)
           TNoise layers f s c0 c1 -> do
             pokeI32 b 0 3 >> pokeI32 b 4 (fromIntegral layers)
             pokeDoubles b 16 (v3l c0) >> pokeDoubles b 40 (v3l c1) >> pokeDoubles b 64 (f : v3l s) >> pure imgNo
           TMarble d f s -> do
             pokeI32 b 0 4 >> pokeDoubles b 64 (v3l d ++ [f] ++ v3l s) >> pure imgNo) 0 (zip [0 ..] texs)
       forM_ (zip [0 ..] motions) $ \(i, (v0, v1)) -> pokeDoubles (pmo `plusPtr` (48 * i)) 0 (v3l v0 ++ v3l v1)
       forM_ (zip [0 ..] frames) $ \(i, r) -> pokeDoubles (pf `plusPtr` (72 * i)) 0 r
       forM_ (zip [0 ..] texels) $ \(i, V3 r g bl) ->
         zipWithM_ (\c x -> pokeByteOff ptx (12 * i + 4 * c) (realToFrac x :: CFloat)) [0 ..] [r, g, bl]
       when needPerlin $ do
         -- Noise.hs:52-92: the reference's permutation tables (embedded below: Graphics.Ray.Noise
         -- does not export them) and the gradients exactly as Noise.hs:88-92 computes them
         -- (randomUnitVector under mkStdGen 666)
         forM_ (zip [0 :: Int ..] [permXTable, permYTable, permZTable]) $ \(a, perm) ->
           zipWithM_ (\j v -> pokeI32 pper (4 * (256 * a + j)) (fromIntegral v)) [0 .. 255] perm
         let grads = evalState (mapM (const randomUnitVector) [1 .. 256 :: Int]) (mkStdGen 666) :: [V3 Double]
         forM_ (zip [0 ..] grads) $ \(j, g) -> pokeDoubles pper (3072 + 24 * j) (v3l g)
       forM_ (zip [0 ..] insts) $ \(i, (b, o, m)) -> do
         let q = pin `plusPtr` (112 * i)
         pokeI32 q 0 b >> pokeI32 q 4 (-1) >> pokeI32 q 8 o >> pokeI32 q 12 0  -- material -1: the leaves' own
         pokeDoubles q 16 (concat m)
       fillBytes sc 0 136
       let arr off n p = pokeI32 sc off (fromIntegral n) >> pokeByteOff sc (off + 8) (if n > 0 then castPtr p else nullPtr :: Ptr ())
       arr 0 (length prims) pp
       arr 16 (length media) pm
       arr 32 (length mats) pmat
       arr 48 nTex pt
       arr 64 (length motions) pmo
       arr 80 (length frames) pf
       arr 96 (length texels) ptx
       pokeByteOff sc 112 (if needPerlin then castPtr pper else nullPtr :: Ptr ())
       arr 120 (length insts) pin
       k (castPtr sc)

-- Noise.hs:52-86 permX / permY / permZ (raytrace_amd/data/perlin_perm.json; the constants of the
-- reference's module, embedded so that the binding asks no change of it)
permXTable :: [Int]
permXTable =
  [ 179, 60, 35, 16, 220, 94, 67, 236, 106, 112, 65, 166, 83, 101, 246, 140, 219, 186, 113, 88, 153, 70, 34, 63
  , 157, 210, 212, 188, 54, 74, 23, 161, 28, 137, 126, 107, 183, 58, 134, 127, 211, 225, 17, 123, 150, 243, 160, 68
  , 75, 239, 173, 221, 89, 109, 61, 72, 159, 80, 154, 18, 214, 144, 197, 24, 105, 32, 84, 226, 136, 29, 139, 97
  , 230, 167, 165, 238, 27, 14, 50, 193, 46, 253, 240, 111, 69, 196, 130, 102, 104, 118, 204, 12, 169, 202, 142, 25
  , 245, 215, 149, 138, 185, 48, 223, 247, 47, 98, 143, 26, 87, 251, 103, 52, 234, 232, 218, 205, 92, 228, 162, 85
  , 122, 191, 242, 164, 129, 192, 255, 231, 147, 91, 178, 213, 176, 36, 120, 155, 241, 222, 177, 20, 152, 141, 51, 171
  , 250, 95, 71, 119, 254, 172, 53, 146, 135, 124, 125, 163, 235, 99, 7, 22, 100, 229, 93, 174, 3, 189, 116, 66
  , 217, 158, 237, 55, 151, 0, 148, 45, 86, 64, 216, 43, 252, 121, 200, 115, 39, 184, 82, 56, 9, 181, 62, 2
  , 81, 209, 44, 79, 19, 110, 41, 10, 194, 15, 132, 224, 249, 96, 233, 117, 49, 203, 5, 37, 11, 59, 168, 114
  , 90, 131, 31, 145, 40, 206, 13, 187, 133, 207, 4, 199, 170, 78, 30, 182, 248, 21, 6, 227, 57, 180, 73, 42
  , 128, 175, 108, 33, 244, 201, 198, 77, 195, 8, 38, 190, 76, 156, 208, 1
  ]

permYTable :: [Int]
permYTable =
  [ 252, 123, 131, 151, 243, 143, 12, 247, 196, 179, 99, 0, 178, 109, 71, 160, 93, 205, 127, 38, 142, 117, 152, 124
  , 166, 95, 200, 121, 15, 17, 10, 190, 116, 158, 173, 75, 248, 191, 197, 58, 70, 184, 226, 146, 6, 239, 165, 113
  , 218, 34, 83, 77, 74, 5, 176, 85, 112, 147, 59, 66, 14, 31, 2, 21, 198, 108, 255, 11, 36, 156, 96, 73
  , 1, 189, 126, 50, 220, 16, 249, 23, 139, 135, 141, 92, 159, 4, 119, 174, 171, 253, 86, 227, 251, 172, 7, 149
  , 207, 212, 224, 44, 187, 91, 175, 84, 28, 211, 180, 195, 52, 98, 244, 125, 138, 54, 210, 201, 209, 219, 133, 240
  , 9, 202, 199, 42, 51, 48, 104, 154, 88, 53, 64, 105, 242, 63, 223, 222, 67, 238, 32, 134, 72, 62, 101, 150
  , 94, 161, 19, 236, 215, 97, 206, 22, 188, 230, 170, 18, 13, 162, 129, 90, 246, 130, 35, 46, 43, 213, 29, 76
  , 241, 61, 30, 136, 235, 87, 114, 68, 183, 177, 250, 132, 3, 122, 110, 145, 81, 78, 232, 69, 60, 80, 216, 65
  , 164, 237, 157, 203, 25, 221, 254, 181, 8, 182, 214, 24, 40, 102, 37, 106, 228, 39, 229, 163, 111, 186, 245, 55
  , 41, 225, 234, 49, 45, 231, 107, 103, 168, 153, 47, 56, 118, 120, 137, 155, 148, 82, 33, 204, 79, 169, 144, 20
  , 27, 128, 192, 217, 100, 208, 115, 140, 233, 89, 193, 185, 167, 57, 26, 194
  ]

permZTable :: [Int]
permZTable =
  [ 153, 90, 163, 138, 20, 136, 79, 100, 93, 38, 185, 31, 193, 43, 161, 2, 30, 37, 87, 6, 127, 207, 96, 51
  , 27, 227, 203, 215, 155, 190, 106, 94, 65, 183, 114, 71, 74, 219, 245, 39, 140, 216, 195, 191, 3, 214, 13, 23
  , 168, 179, 218, 133, 102, 53, 194, 124, 166, 108, 116, 246, 35, 109, 220, 121, 205, 110, 83, 242, 252, 231, 25, 128
  , 61, 57, 187, 222, 189, 228, 148, 101, 239, 162, 48, 150, 55, 174, 178, 42, 200, 160, 58, 206, 11, 92, 204, 67
  , 8, 113, 34, 172, 181, 177, 66, 16, 243, 159, 197, 135, 249, 241, 28, 147, 158, 139, 176, 88, 29, 149, 254, 226
  , 192, 201, 202, 186, 69, 45, 72, 199, 107, 99, 209, 10, 230, 217, 247, 89, 50, 129, 15, 64, 248, 167, 180, 146
  , 210, 169, 4, 81, 97, 238, 5, 237, 125, 236, 95, 9, 104, 221, 32, 86, 165, 134, 224, 182, 198, 234, 253, 59
  , 164, 52, 60, 208, 103, 22, 46, 188, 54, 12, 1, 112, 144, 137, 47, 156, 98, 78, 18, 82, 175, 225, 19, 184
  , 244, 49, 120, 157, 130, 70, 80, 251, 212, 250, 119, 118, 196, 223, 105, 68, 84, 21, 145, 173, 56, 235, 91, 17
  , 126, 76, 131, 117, 152, 111, 33, 36, 233, 141, 122, 85, 7, 123, 44, 62, 115, 26, 0, 40, 229, 211, 213, 63
  , 143, 77, 14, 24, 142, 154, 73, 132, 171, 41, 170, 240, 75, 151, 232, 255
  ]

-- | cs_background restricted to what the device evaluates: (1 - a) c0 + a c1 with
-- a = (y + 1) / 2 (`const c` is c0 = c1; test/Main.hs's `sky` and `grayFade`).  The closure is
-- probed at 26 unit directions and 3 origins; any disagreement (> 1e-12 relative) sends the
-- whole render to the CPU path.
reifyBackground :: (Ray -> Color) -> Maybe (Int32, Color, Color)
reifyBackground bg =
  let c0 = bg (Ray (V3 0 0 0) (V3 0 (-1) 0))
      c1 = bg (Ray (V3 0 0 0) (V3 0 1 0))
      dirs = [ d | x <- [-1, 0, 1], y <- [-1, 0, 1], z <- [-1, 0, 1], let v = V3 x y z, norm v > 0, let d = v / pure (norm v) ]
      origins = [V3 0 0 0, V3 3 (-2) 7, V3 (-500) 250 1000]
      expect (V3 _ y _) = let a = 0.5 * (y + 1) in pure (1 - a) * c0 + pure a * c1
      close p q = and (zipWith (\u w -> abs (u - w) <= 1e-12 * (1 + abs w)) (v3l p) (v3l q))
      ok = and [ close (bg (Ray o d)) (expect d) | o <- origins, d <- dirs ]
  in if ok then Just (if close c0 c1 then 0 else 1, c0, c1) else Nothing

withCamera :: R.CameraSettings -> (Int32, Color, Color) -> (Ptr RtCamera -> IO a) -> IO a
withCamera R.CameraSettings{..} (bgKind, c0, c1) k =
  let targets = cs_redirectTargets
  in allocaBytes (max 1 (80 * length targets)) $ \pt ->
     allocaBytes 184 $ \p -> do
       forM_ (zip [0 ..] targets) $ \(i, (prob, q, u, v)) ->
         pokeDoubles (pt `plusPtr` (80 * i)) 0 (prob : v3l q ++ v3l u ++ v3l v)
       fillBytes p 0 184
       pokeDoubles p 0 (v3l cs_center ++ v3l cs_lookAt ++ v3l cs_up ++ [cs_vfov, cs_aspectRatio])
       pokeI32 p 88 (fromIntegral cs_imageWidth)
       pokeI32 p 92 (fromIntegral cs_samplesPerPixel)
       pokeI32 p 96 (fromIntegral cs_maxRecursionDepth)
       pokeI32 p 100 bgKind
       pokeDoubles p 104 (v3l c0 ++ v3l c1 ++ [cs_defocusAngle, cs_focusDist])
       pokeI32 p 168 (fromIntegral (length targets))
       pokeByteOff p 176 (if null targets then nullPtr else castPtr pt :: Ptr ())
       k (castPtr p)

data Precision = Binary64 | Float32
  deriving (Eq, Show)

-- | Devices and precision of a render.  The default renders in binary64 (the reference's
-- arithmetic) on every visible GPU, rows dealt to them round-robin (rt_exec device list).
data DeviceOptions = DeviceOptions
  { doDevices :: Maybe [Int]      -- ^ Nothing: every visible device
  , doPrecision :: Precision
  , doRowBlock :: Int
  }

defaultDeviceOptions :: DeviceOptions
defaultDeviceOptions = DeviceOptions Nothing Binary64 1

data RenderError
  = NotReifiable                  -- ^ the scene, a material, a texture or the background is a closure
  | LibraryError Int String       -- ^ an RT_E_* code and rt_last_error's message
  deriving (Show)

-- | The 8-bit transfer of the reference's writers: 'SRGB' = writeImage, 'Sqrt' = writeImageSqrt
-- (Ray.hs:248-260); rt.h RT_EXEC_ENCODE8_SRGB / RT_EXEC_ENCODE8_SQRT.
data Encoding = SRGB | Sqrt
  deriving (Eq, Show)

-- | Number of visible HIP devices (0 when there is none).
deviceCount :: IO Int
deviceCount = (\n -> if n > 0 then fromIntegral n else 0) <$> c_rt_device_count

withExec :: DeviceOptions -> Maybe Encoding -> [Int] -> (Ptr RtExec -> IO a) -> IO a
withExec DeviceOptions{..} enc devs k =
  withArray (map fromIntegral devs :: [Int32]) $ \pd ->
  allocaBytes 32 $ \p -> do
    fillBytes p 0 32
    pokeI32 p 0 (fromIntegral (if null devs then 0 else head devs))
    pokeI32 p 4 1                                              -- n_shards: the whole image
    pokeI32 p 8 0
    pokeI32 p 12 (fromIntegral (max 1 doRowBlock))
    let flags = (if doPrecision == Float32 then 1 else 0)     -- RT_EXEC_F32
              + (case enc of Nothing -> 0; Just SRGB -> 2; Just Sqrt -> 4)  -- RT_EXEC_ENCODE8_*
    pokeI32 p 16 flags
    pokeI32 p 20 (fromIntegral (length devs))
    pokeByteOff p 24 (castPtr pd :: Ptr ())
    k (castPtr p)

-- | The device's Philox key for a StdGen: a splitmix digest of the generator's (seed, gamma),
-- the same derivation as raytrace_amd.core.StdGen.key (so both hosts render the same image).
philoxKey :: StdGen -> Word64
philoxKey g = let (seed, gamma) = unseedSMGen (unStdGen g) in mix64 (seed `xor` mix64 gamma)
  where
    mix64 z0 = let z1 = (z0 `xor` (z0 `shiftR` 33)) * 0xff51afd7ed558ccd
                   z2 = (z1 `xor` (z1 `shiftR` 33)) * 0xc4ceb9fe1a85ec53
               in z2 `xor` (z2 `shiftR` 33)

-- | One rt_render call into a fresh ForeignPtr of h x w elements of 3 `elem`s each: the scene
-- flattened (shared transformed objects instanced), the camera reified, the device list resolved.
renderRaw :: Storable e => DeviceOptions -> Maybe Encoding -> R.CameraSettings -> Geometry m Material -> StdGen
          -> (Int -> IO (ForeignPtr e)) -> IO (Either RenderError (Int, Int, ForeignPtr e))
renderRaw opts enc settings world gen alloc =
  case (geoDesc world, reifyBackground (R.cs_background settings)) of
    (Just desc, Just bg) -> do
      tagged <- tagShared desc
      case flatten tagged of
        Nothing -> pure (Left NotReifiable)
        Just flat -> do
          devs <- case doDevices opts of
            Just ds -> pure ds
            Nothing -> (\n -> [0 .. max 1 n - 1]) <$> deviceCount
          withCamera settings bg $ \cam ->
            withFlatScene flat $ \sc ->
            withExec opts enc devs $ \ex -> do
              h <- fromIntegral <$> c_rt_image_height cam
              let w = R.cs_imageWidth settings
              if h <= 0 || w <= 0 then pure (Left (LibraryError (-2) "empty image")) else do
                fp <- alloc (3 * h * w)
                rc <- withForeignPtr fp $ \out -> c_rt_render cam sc (philoxKey gen) ex (castPtr out) nullPtr
                if rc /= 0
                  then Left . LibraryError (fromIntegral rc) <$> (c_rt_last_error >>= peekCString)
                  else pure (Right (h, w, fp))
    _ -> pure (Left NotReifiable)

-- | Render on the GPU through rt_render.  The output buffer is a ForeignPtr that becomes the
-- storable (S) massiv matrix directly: no copy, no list (binary64); the FP32 path widens the
-- floats in one pass over the buffer.
renderOnDevice :: DeviceOptions -> R.CameraSettings -> Geometry m Material -> StdGen
               -> IO (Either RenderError (A.Matrix A.S Color))
renderOnDevice opts settings world gen
  | doPrecision opts == Binary64 = do
      r <- renderRaw opts Nothing settings world gen (\n -> mallocForeignPtrArray n :: IO (ForeignPtr CDouble))
      pure (fmap (\(h, w, fp) -> asColors h w (castForeignPtr fp)) r)
  | otherwise = do
      r <- renderRaw opts Nothing settings world gen (\n -> mallocForeignPtrArray n :: IO (ForeignPtr CFloat))
      case r of
        Left e -> pure (Left e)
        Right (h, w, fp32) -> do
          let n = 3 * h * w
          fp <- mallocForeignPtrArray n :: IO (ForeignPtr CDouble)
          withForeignPtr fp32 $ \src -> withForeignPtr fp $ \dst ->
            forM_ [0 .. n - 1] $ \i -> peekElemOff src i >>= pokeElemOff dst i . realToFrac
          pure (Right (asColors h w (castForeignPtr fp)))
  where
    -- V3 Double is stored as 3 contiguous doubles (linear's Storable instance)
    asColors h w fp = A.resize' (A.Sz2 h w) (AU.unsafeArrayFromForeignPtr0 A.Par (fp :: ForeignPtr Color) (A.Sz1 (h * w)))

-- | The 8-bit codes writeImage / writeImageSqrt would store for the render, encoded on the GPU
-- right after the gather (rt.h RT_EXEC_ENCODE8_*): h x w (R, G, B) bytes, bit-identical to
-- encoding the linear render.
renderImage8 :: DeviceOptions -> Encoding -> R.CameraSettings -> Geometry m Material -> StdGen
             -> IO (Either RenderError (A.Matrix A.S (V3 Word8)))
renderImage8 opts enc settings world gen = do
  r <- renderRaw opts (Just enc) settings world gen (\n -> mallocForeignPtrBytes n :: IO (ForeignPtr Word8))
  pure (fmap (\(h, w, fp) -> A.resize' (A.Sz2 h w)
                (AU.unsafeArrayFromForeignPtr0 A.Par (castForeignPtr fp :: ForeignPtr (V3 Word8)) (A.Sz1 (h * w)))) r)

-- | Render and write the image file in one step: @raytraceToFile SRGB path cs world gen@ writes
-- what @writeImage path (raytrace cs world gen)@ writes (Sqrt: writeImageSqrt), with the 8-bit
-- encoding done on the GPU; scenes the device cannot render go through the reference's CPU
-- raytrace and writer.
raytraceToFile :: R.ToRandom m => Encoding -> FilePath -> R.CameraSettings -> Geometry m Material
               -> StdGen -> IO ()
raytraceToFile enc path settings world gen = do
  r <- renderImage8 defaultDeviceOptions enc settings world gen
  case r of
    Right codes -> I.writeImageAuto path (A.map toPixel codes)
    Left e | fallback e -> (if enc == SRGB then R.writeImage else R.writeImageSqrt) path
                             (R.raytrace settings (toReferenceRandom world) gen)
           | otherwise -> ioError (userError ("Graphics.Ray.Device.raytraceToFile: " ++ show e))
  where
    -- the codes are already the stored 8-bit values: written as non-linear sRGB bytes, unconverted
    toPixel :: V3 Word8 -> C.Pixel (SRGB 'NonLinear) Word8
    toPixel (V3 r g b) = C.Pixel (C.ColorSRGB r g b)

-- | Library results that send a render to the reference's CPU path: a closure somewhere in the
-- scene, RT_E_UNSUPPORTED (e.g. a non-Euclidean transform) and RT_E_STACK (a hierarchy deeper
-- than the device's traversal stack).
fallback :: RenderError -> Bool
fallback NotReifiable = True
fallback (LibraryError code _) = code == -3 || code == -5

-- | 'Graphics.Ray.raytrace' on the GPU: same arguments, same result (Ray.hs:121-238).  Falls
-- back to the reference's CPU path when the scene is not reifiable or the library reports
-- RT_E_UNSUPPORTED or RT_E_STACK; any other library error (no device, a HIP failure) is raised.
-- The signature is the reference's (Ray.hs:121): the CPU fallback lifts the geometry into
-- 'State StdGen' through 'R.toRandom' ('toReferenceRandom') instead of mapping inside @m@.
raytrace :: R.ToRandom m => R.CameraSettings -> Geometry m Material -> StdGen -> A.Matrix A.D Color
raytrace = raytraceWith defaultDeviceOptions

raytraceWith :: R.ToRandom m => DeviceOptions -> R.CameraSettings -> Geometry m Material -> StdGen
             -> A.Matrix A.D Color
raytraceWith opts settings world gen =
  case unsafePerformIO (renderOnDevice opts settings world gen) of
    Right img -> A.delay img
    Left e | fallback e -> R.raytrace settings (toReferenceRandom world) gen
           | otherwise -> error ("Graphics.Ray.Device.raytrace: rt_render failed: " ++ show e)
{-# NOINLINE raytraceWith #-}
