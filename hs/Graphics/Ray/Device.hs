{-# LANGUAGE ForeignFunctionInterface #-}
{-# LANGUAGE RecordWildCards #-}
-- | GPU drop-in for 'Graphics.Ray.raytrace' (reference: src/Graphics/Ray.hs:121-238).
--
-- SOURCE ONLY: GHC is not available in the build container, so this module is not compiled or
-- tested here; the C ABI it binds (include/rt.h) is exercised from Python/ctypes and C by
-- tests/.  It is the binding a maintainer of UnaryPlus/raytrace would add (INTEGRATION.md).
--
-- The reference's 'Geometry', 'Material', 'Texture' and background are closures, so the
-- device path needs a deep embedding: 'Scene' mirrors the smart constructors (same names with
-- a D suffix), 'flatten' bakes it into the rt_prim / rt_medium / rt_material / rt_texture
-- records of include/rt.h, and 'raytraceDevice' calls rt_render.  'toGeometry' rebuilds the
-- reference closure from the same description, so a program can keep calling the CPU
-- 'raytrace' when the device answers RT_E_UNSUPPORTED.
module Graphics.Ray.Device
  ( Scene(..), MaterialD(..), TextureD(..), BackgroundD(..)
  , raytraceDevice, raytraceAuto, toGeometry
  ) where

import Graphics.Ray
import Linear (V3(V3), M44)
import Data.Word (Word64)
import Data.Int (Int32, Int64)
import Foreign
import Foreign.C.Types
import Foreign.C.String (CString, peekCString)
import System.IO.Unsafe (unsafePerformIO)
import qualified Data.Massiv.Array as A
import qualified Data.Massiv.Array.Unsafe as AU
import Control.Monad.State (State)

-- | Reified textures (Texture.hs:18-78).  Images are row-major linear RGB (row 0 at the top);
-- noise / marble textures make the flattened scene carry the Perlin tables (rt_perlin:
-- permX / permY / permZ and Noise.hs's `gradients`).
data TextureD
  = ConstantD Color | CheckerD Int Int Color Color
  | ImageD (A.Matrix A.U Color)
  | NoiseD Int Double (V3 Double) Color Color     -- ^ layers, frequency, shift, colour 0, colour 1
  | MarbleD Vec3 Double (V3 Double)               -- ^ stripe direction, frequency, shift

-- | Reified materials (Material.hs:41-129).
data MaterialD
  = LightSourceD TextureD | PitchBlackD | LambertianD TextureD | LommelSeeligerD TextureD
  | MirrorD TextureD | MetalD Double TextureD | DielectricD Double | TransparentD TextureD
  | IsotropicD TextureD | AnisotropicD Double TextureD

-- | Reified backgrounds: `const c` and the y-lerps `sky` / `grayFade` of test/Main.hs:19-28.
data BackgroundD = ConstBG Color | LerpYBG Color Color

-- | Deep embedding of Geometry.hs's constructors.
data Scene
  = SphereD Point3 Double
  | ParallelogramD Point3 Vec3 Vec3
  | TriangleD (Point3, V2D) (Point3, V2D) (Point3, V2D)
  | GroupD [Scene]
  | BvhTreeD [Scene]
  | TransformD (M44 Double) Scene
  | MovingD Vec3 Vec3 Scene
  | MediumD Double Scene
  | WithMaterialD MaterialD Scene        -- ^ `material <$ geometry`
type V2D = (Double, Double)

-- ---------------------------------------------------------------- C ABI (include/rt.h)

data RtScene
data RtCamera
data RtExec
data RtStats

foreign import ccall safe "rt_render"
  c_rt_render :: Ptr RtCamera -> Ptr RtScene -> Word64 -> Ptr RtExec -> Ptr CFloat -> Ptr RtStats -> IO CInt
foreign import ccall unsafe "rt_last_error"
  c_rt_last_error :: IO CString
foreign import ccall unsafe "rt_image_height"
  c_rt_image_height :: Ptr RtCamera -> IO CInt

-- | Render on the GPU.  Left carries the library's message (RT_E_UNSUPPORTED means "use the
-- CPU 'raytrace'"); Right is the h x w matrix of linear colours (row 0 at the top), each the
-- mean of cs_samplesPerPixel samples — the value Ray.hs:238 computes.
raytraceDevice :: CameraSettings -> BackgroundD -> Scene -> Word64 -> Either (Int, String) (A.Matrix A.S Color)
raytraceDevice settings bg scene seed = unsafePerformIO $
  withCamera settings bg $ \cam ->
  withFlatScene scene $ \sc ->
  withExec $ \ex -> do
    h <- fromIntegral <$> c_rt_image_height cam
    let w = cs_imageWidth settings
    allocaArray (h * w * 3) $ \out -> do
      rc <- c_rt_render cam sc seed ex out nullPtr
      if rc /= 0
        then do msg <- c_rt_last_error >>= peekCString
                pure (Left (fromIntegral rc, msg))
        else do xs <- peekArray (h * w * 3) out
                let px k = let b = 3 * k in V3 (realToFrac (xs !! b)) (realToFrac (xs !! (b + 1))) (realToFrac (xs !! (b + 2)))
                pure (Right (A.makeArray A.Seq (A.Sz (h A.:. w)) (\(j A.:. i) -> px (j * w + i))))

-- | GPU when the scene is reifiable, otherwise the reference's CPU path.
raytraceAuto :: CameraSettings -> BackgroundD -> Scene -> Word64 -> StdGen -> A.Matrix A.D Color
raytraceAuto settings bg scene seed gen =
  case raytraceDevice settings bg scene seed of
    Right m -> A.delay m
    Left _ -> raytrace settings { cs_background = background bg } (toGeometry scene) gen
  where
    background (ConstBG c) = const c
    background (LerpYBG c0 c1) = \(Ray _ (V3 _ y _)) -> let a = 0.5 * (y + 1) in (1 - a) *^^ c0 + a *^^ c1
    s *^^ V3 x y z = V3 (s * x) (s * y) (s * z)

-- | The reference closure for the same description (CPU fallback and cross-checks).
toGeometry :: Scene -> Geometry (State StdGen) Material
toGeometry = error "toGeometry: build with the reference constructors (sphere, parallelogram, group, bvhTree, transform, moving, constantMedium, (<$)); see INTEGRATION.md"

-- Marshalling helpers (flattening mirrors raytrace_amd/scene.py: rigid transforms baked into
-- the leaves, outermost `<$` wins, media lifted to the top level, depth-first `order` kept).
withCamera :: CameraSettings -> BackgroundD -> (Ptr RtCamera -> IO a) -> IO a
withCamera = error "marshal rt_camera_settings (layout: include/rt.h)"

withFlatScene :: Scene -> (Ptr RtScene -> IO a) -> IO a
withFlatScene = error "marshal rt_scene (layout: include/rt.h; reference implementation: raytrace_amd/scene.py)"

withExec :: (Ptr RtExec -> IO a) -> IO a
withExec k = allocaBytes 24 $ \p -> do
  pokeByteOff p 0 (0 :: Int32)   -- device
  pokeByteOff p 4 (1 :: Int32)   -- n_shards
  pokeByteOff p 8 (0 :: Int32)   -- shard
  pokeByteOff p 12 (4 :: Int32)  -- row_block
  pokeByteOff p 16 (0 :: Int32)  -- flags
  pokeByteOff p 20 (0 :: Int32)
  k (castPtr p)
